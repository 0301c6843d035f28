# Round 5 batch 1: full GPU suite after the data-path split + wire framing, then the bench (incl. configs 4 / 5).
cd $GRAFT_REPO_ROOT
out=gpurun_out/b1
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $out/gpu_tests.log 2>&1
rc=$?
tail -15 $out/gpu_tests.log
# 0 = passed, 1 = some tests failed: the GPU is fine, measure; anything else (timeout, crash): stop here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python bench.py > $out/bench.json 2> $out/bench.err
brc=$?
tail -c 1500 $out/bench.json
exit $(( rc != 0 ? rc : brc ))
