#!/bin/bash
# GPU driver: one parameterised script for every experiment (replaces the per-experiment one-offs).
#   tools/gpu.sh TAG STEP [STEP ...]
# STEP is one of
#   pytest:<file[,file...]>     pytest -m gpu on those test files (tests/ prefix implied)
#   smoke                       __graft_entry__.smoke()
#   pytestall                   the whole GPU suite
#   rocm:<lib|intree>[:k]       tools/rocm_rate.py (torch_rocm stream, 7B bf16) on a build
#   bench[:args]                bench.py with comma-separated extra args
#   ubench:<name>               tools/ubench/<name>
#   py:<script>[:args]          python tools/<script> with comma-separated args
#   sh:<script>                 bash tools/<script> (environment passed through)
#   ab:<lib|intree>[,<lib>...]  tools/ab_apply.py on those builds (AB_* environment)
# Every GPU step runs under its own timeout; the first failing step ends the script.
# Before any step, libfks.so and the oracle are compiled from the pushed sources: the
# objects and build/ are not pushed (.gpurunignore), so make rebuilds them on the box and
# relinks libfks.so; the log records the build id the run then loads.
set -o pipefail
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
echo "[$TAG] build: make -C fate-llm_amd, make -C oracle -> $OUT/00_build.log"
{ timeout -k 10 600 make -j16 -C fate-llm_amd && timeout -k 10 120 make -C oracle; } > "$OUT/00_build.log" 2>&1 \
  || { tail -20 "$OUT/00_build.log"; echo "[$TAG] build failed"; exit 3; }
python -c "import ctypes; l = ctypes.CDLL('fate-llm_amd/python/fate_llm/algo/fedkseed/libfks.so'); \
l.fks_build_id.restype = ctypes.c_char_p; print('fks_build_id', l.fks_build_id().decode())" | tee -a "$OUT/00_build.log"
grep -c 'hipcc.*fks_device.hip' "$OUT/00_build.log" | sed -e 's/^/device objects compiled on this box: /' | tee -a "$OUT/00_build.log"
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  arg=${step#*:}
  [ "$arg" = "$step" ] && arg=""
  log="$OUT/$(printf %02d $n)_${kind}.log"
  echo "[$TAG] step $n: $step -> $log"
  case $kind in
    pytest)
      files=$(echo "$arg" | tr ',' ' ' | sed -e 's#\([^ ]*\)#tests/\1#g')
      timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $files > "$log" 2>&1 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 ;;
    pytestall)
      timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > "$log" 2>&1 ;;
    rocm)
      lib=${arg%%:*}
      k=${arg#*:}
      [ "$k" = "$arg" ] && k=64
      if [ "$lib" = intree ]; then
        timeout -k 10 300 python -u tools/rocm_rate.py --ref-seeds 0 --modes torch_rocm --k "$k" > "$log" 2>&1
      else
        FKS_LIB_OVERRIDE=$lib timeout -k 10 300 python -u tools/rocm_rate.py --ref-seeds 0 --modes torch_rocm --k "$k" > "$log" 2>&1
      fi ;;
    bench)
      timeout -k 10 600 python -u bench.py $(echo "$arg" | tr ',' ' ') > "$log" 2>&1 ;;
    ubench)
      timeout -k 10 300 "tools/ubench/$arg" > "$log" 2>&1 ;;
    py)
      script=${arg%%:*}
      a=${arg#*:}
      [ "$a" = "$arg" ] && a=""
      timeout -k 10 900 python -u "tools/$script" $(echo "$a" | tr ',' ' ') > "$log" 2>&1 ;;
    sh)
      timeout -k 10 1200 bash "tools/$arg" > "$log" 2>&1 ;;
    ab)
      timeout -k 10 600 python -u tools/ab_apply.py $(echo "$arg" | tr ',' ' ') > "$log" 2>&1 ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  tail -3 "$log"
  if [ $rc -ne 0 ]; then
    echo "[$TAG] step $n failed rc=$rc"
    exit $rc
  fi
done
