# First-round GPU session: parity tests, then the lanes-per-packet exploration.
set -u
mkdir -p gpurun_out
make -C oracle -s
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider > gpurun_out/pytest1.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -15 gpurun_out/pytest1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python scripts/explore.py --cfg 2,5,3 --reps 5 > gpurun_out/explore1.log 2>&1
rc=$?
echo "explore rc=$rc"
grep -v amdgpu.ids gpurun_out/explore1.log | tail -50
exit $rc
