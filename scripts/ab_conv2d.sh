# Same-box A/B of two extension builds on the trunk conv microbenchmark
# (_C_head.so / _C_new.so at the repo root, see ab_so.sh):
#   gpurun -- 'bash scripts/ab_conv2d.sh [conv_bench args]'
set -e
for k in 1 2; do
 for v in head new; do cp _C_$v.so ncnet_amd/_C.so; echo "== $v"; timeout -k 10 120 python -u scripts/conv_bench.py "$@" 2>&1 | grep -v amdgpu; done
done
