# round 5: C4 at full size -- the 70B fp32 K=4096 reconstruct (8 chunks), timed, then
# tools/c4_70b.py --verify: the embed prefix record (replayed through the oracle by
# tests/test_c4_fullsize_record.py) and a chunk boundary recomputed by one call
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05e
bash tools/gpu.sh r05e_build pytest:test_gpu_selfcheck.py || exit $?
timeout -k 10 1000 python -u tools/c4_70b.py --ks 4096 --progress --verify gpurun_out/r05e/r05_c4_verify.npz \
  > gpurun_out/r05e/r05_c4_70b_fp32_k4096.log 2>&1
rc=$?
tail -3 gpurun_out/r05e/r05_c4_70b_fp32_k4096.log
exit $rc
