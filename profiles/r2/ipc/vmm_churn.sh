#!/bin/bash
# vmm_churn_probe (csrc/tools/vmm_churn_probe.hip) against /opt/rocm's and PyTorch's bundled HIP runtime.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/vmmchurn
mkdir -p $OUT
hipcc --offload-arch=gfx950 -O2 -std=c++20 csrc/tools/vmm_churn_probe.hip -o /tmp/vmmchurn || exit 1
TL=$(python -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
mkdir -p /tmp/tl && ln -sf "$TL/libamdhip64.so" /tmp/tl/libamdhip64.so.7
for rt in opt torch; do
  if [ $rt = torch ]; then export LD_LIBRARY_PATH=/tmp/tl:$TL; else unset LD_LIBRARY_PATH; fi
  for fv in 1 0; do
    timeout -k 5 120 /tmp/vmmchurn 150 3 $fv > $OUT/${rt}_freeva$fv.log 2>&1
    rc=$?
    echo "$rt free_va=$fv rc=$rc: $(tail -1 $OUT/${rt}_freeva$fv.log)"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done
exit 0
