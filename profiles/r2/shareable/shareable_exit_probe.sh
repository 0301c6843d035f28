cd $GRAFT_REPO_ROOT
for v in plain del_tensor del_pool leak; do echo "== $v"; timeout -k 5 120 python profiles/r2/shareable/shareable_exit_probe.py $v 2>&1 | grep -v amdgpu.ids | tail -25; echo "rc=$?"; done
