export TUNE='[{"RTW_SHADE_MIN":"48","RTW_WAVES":"6"}]'
for lib in "" build/rtw_ablate_rng.so build/rtw_ablate_math.so build/rtw_ablate_both.so; do
  echo "lib=$lib"; RTW_LIB=$lib timeout -k 10 200 python tools/tune.py 100 || exit $?
done
