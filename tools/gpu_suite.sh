#!/bin/bash
# The full GPU suite and smoke(), as the driver runs them at round end.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r02o}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 97; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 98; }
tail -1 gpurun_out/${TAG}_smoke.log
