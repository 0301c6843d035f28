# one-off GPU batch (round 6): the new staging / path tests, the runtime race reproducer's mixed mode
mkdir -p gpurun_out/r6b gpurun_out/race
timeout -k 10 700 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -x -v -s --timeout 300 --timeout-method thread \
  -k "reference_framing_staging or above_arena or staging_bounded_by_segment" > gpurun_out/r6b/staging.log 2>&1
rc=$?; echo "staging rc=$rc" > gpurun_out/r6b/rcs.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 5 60 ./pccl_amd/lib/pccl_stream_race mixed_null 20 8 8 > gpurun_out/race/mixed_null.json 2> gpurun_out/race/mixed_null.err
echo "mixed_null rc=$?" >> gpurun_out/race/rcs.txt
