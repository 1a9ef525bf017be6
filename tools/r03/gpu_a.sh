#!/bin/bash
# round-3 GPU call A: the new parity tests (multi-block slice chunks, full size at wd 0.0,
# stream ordering), the smoke, the CPU share of the box, the default bench line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
python3 -c "
import os, sys; sys.path.insert(0, '.')
import bench
print('nproc', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)), 'usable', bench.usable_cpus())
for f in ('/sys/fs/cgroup/cpu.max', '/sys/fs/cgroup/cpu/cpu.cfs_quota_us'):
    try: print(f, open(f).read().strip())
    except OSError as e: print(f, e)
print('OMP_NUM_THREADS', os.environ.get('OMP_NUM_THREADS'))
" > gpurun_out/r03a_cpus.log 2>&1
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_streams.py tests/test_gpu_slice.py tests/test_gpu_fullsize.py tests/test_gpu_wincache.py \
  tests/test_gpu_optimizer_kseed.py > gpurun_out/r03a_pytest.log 2>&1 || { tail -30 gpurun_out/r03a_pytest.log; exit 91; }
tail -3 gpurun_out/r03a_pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03a_smoke.log 2>&1 || { tail gpurun_out/r03a_smoke.log; exit 92; }
tail -1 gpurun_out/r03a_smoke.log
timeout -k 10 300 python3 -u bench.py > gpurun_out/r03a_bench.log 2>&1 || { tail gpurun_out/r03a_bench.log; exit 93; }
tail -1 gpurun_out/r03a_bench.log
