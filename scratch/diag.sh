set -u
for order in torch_first lib_first; do
  timeout -k 10 120 python scratch/diag_runtime.py $order 2>&1 | grep -v amdgpu.ids; echo "rc=$?"
  ROCE_ICRC_LIB=/root/repo/scratch/libroceicrc_cov5.so timeout -k 10 120 python scratch/diag_runtime.py $order 2>&1 | grep -v amdgpu.ids; echo "rc=$?"
done
