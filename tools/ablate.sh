# timing-only ablation builds (wrong images by construction) -- see csrc/Makefile `ablate`/`stamps`
export TUNE='[{"bvh":"sah"}]'
for lib in "" build/rtw_ablate_rng.so build/rtw_ablate_math.so build/rtw_ablate_reject.so build/rtw_ablate_both.so; do
  echo "lib=$lib"; RTW_LIB=$lib timeout -k 10 200 python tools/tune.py 100 || exit $?
done
for lib in build/rtw_stamps.so build/rtw_stamps_reject.so build/rtw_stamps_rng.so; do
  echo "stamps lib=$lib"; RTW_LIB=$lib timeout -k 10 120 python tools/stamps.py 20 || exit $?
done
