#!/bin/bash
# Full GPU suite, then the round's measurement set (tools/profile_round.sh) under $TAG.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r02h}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 97; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
TAG=$TAG timeout -k 10 900 bash tools/profile_round.sh || exit $?
