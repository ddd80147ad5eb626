set -u
for U in 2 8; do
echo "U=$U"
ROCE_ICRC_LIB=$PWD/scratch/libroceicrc_u$U.so timeout -k 10 200 python scripts/explore.py --cfg 2,3 --reps 5 --lanes 4,8,16 2>&1 | grep -v amdgpu.ids
done
