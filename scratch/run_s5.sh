set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2 || exit 1
echo "== spin"; timeout -k 10 120 python scripts/latency.py 2>&1 | grep call || exit 1
