set -u
make -C oracle -s
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider 2>&1 | tail -3
rc=${PIPESTATUS[0]}; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/explore.py --cfg 2,5,3 --reps 5 --lanes 2,4,8,16 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python scratch/sustain.py 2>&1 | grep -v amdgpu.ids
