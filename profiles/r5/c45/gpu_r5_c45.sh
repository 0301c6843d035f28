set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c45
timeout -k 10 200 python benchmarks/fault_tolerance.py --transport tcp --peers 8 --mib 1024 --log-dir gpurun_out/c45/ft_tcp > gpurun_out/c45/ft_tcp.json 2> gpurun_out/c45/ft_tcp.err && \
timeout -k 10 150 python benchmarks/fault_tolerance.py --transport ipc --peers 8 --mib 1024 --log-dir gpurun_out/c45/ft_ipc > gpurun_out/c45/ft_ipc.json 2> gpurun_out/c45/ft_ipc.err && \
timeout -k 10 150 python benchmarks/shared_state_sync.py --transport tcp --params 1e9 > gpurun_out/c45/ss_tcp.json 2> gpurun_out/c45/ss_tcp.err && \
timeout -k 10 150 python benchmarks/shared_state_sync.py --transport ipc --params 1e9 > gpurun_out/c45/ss_ipc.json 2> gpurun_out/c45/ss_ipc.err
rc=$?
cat gpurun_out/c45/*.json
exit $rc
