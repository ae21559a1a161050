# same-box A/B of library builds x env knobs (tools/tune.py, C2 at reduced spp)
SPP=${SPP:-100}
CFG=${CFG:-c2}
for lib in ${LIBS:-default}; do
  echo "lib=$lib"
  if [ "$lib" = default ]; then lib=""; fi
  RTW_LIB=$lib timeout -k 10 300 python tools/tune.py $SPP $CFG || exit $?
done
