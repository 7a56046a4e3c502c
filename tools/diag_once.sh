set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 120 python tools/run_workload.py tests/golden/workloads/qos_mix.yaml 500Nodes --check
