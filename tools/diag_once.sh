set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_framework.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
timeout -k 10 300 python -u bench.py --no-cpu --no-config3 --steps 2 --warmup 1 > gpurun_out/bench_scan.log 2>&1 || { tail -20 gpurun_out/bench_scan.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_scan.log').read().splitlines()[-1]);print(d['scan'])"
