# Round 6 session e: the compact kernel with the output ring (16 rounds,
# 8-group turns, sc1): ragged / golden / parity / C-ABI / receive tests, then
# the ACK evidence set (bench line, rocprof summary, PMC traffic).
TESTS="tests/test_gpu_tiny.py tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_capi.py tests/test_gpu_recv.py" \
  bash scripts/gpu_session.sh r06e ack
