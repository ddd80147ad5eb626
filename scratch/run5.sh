set -u
make -C oracle -s
timeout -k 10 400 python -m pytest tests -m gpu -q -x -p no:cacheprovider 2>&1 | tail -3
rc=${PIPESTATUS[0]}; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/explore.py --cfg 2,3 --reps 5 --lanes 2,4,8,16 2>&1 | grep -v amdgpu.ids
