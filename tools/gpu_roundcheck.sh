#!/bin/bash
# The driver's round-end GPU tiers, rehearsed (repo root on the GPU box): the whole
# -m gpu suite, __graft_entry__.smoke(), and the default bench line.
#   bash tools/gpu_roundcheck.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r02}
timeout -k 10 900 python3 -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_gpu_pytest.log 2>&1 || { tail -40 gpurun_out/${tag}_gpu_pytest.log; exit 95; }
tail -3 gpurun_out/${tag}_gpu_pytest.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.log 2>&1 \
  || { tail -20 gpurun_out/${tag}_smoke.log; exit 96; }
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 97; }
tail -1 gpurun_out/${tag}_bench.log
