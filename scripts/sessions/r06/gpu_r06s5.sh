# Round 6: the sorted kernel's range tests on the shipped library, then cfg5
# knob A/B on the current small kernel (tail share, flush policy, waves).
set -u
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sorted.py > $O/pytest_sorted_r06s5.log 2>&1
rc=$?; tail -16 $O/pytest_sorted_r06s5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u scratch/bench_ab.py --workloads cfg5 --rounds 3 scratch/libs/cur.so scratch/libs/s5tail8.so scratch/libs/s5tail32.so scratch/libs/s5pol2.so scratch/libs/s5w10.so > $O/ab_r06s5.txt 2>&1
rc=$?; cat $O/ab_r06s5.txt; exit $rc
