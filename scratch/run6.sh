set -u
timeout -k 10 200 python scripts/explore.py --cfg 5 --reps 5 --lanes 1,2,4,8 2>&1 | grep -v amdgpu.ids
ROCE_ICRC_LIB=$PWD/scratch/libroceicrc_ablate.so timeout -k 10 200 python scripts/explore.py --cfg 5 --reps 5 --lanes 1,2,4,8 2>&1 | grep -v amdgpu.ids
