# Same-box A/B of two builds of the extension (box-to-box clock spread is
# larger than most kernel changes): build HEAD and the working tree, copy them
# to _C_head.so / _C_new.so at the repo root, then
#   gpurun -- 'bash scripts/ab_so.sh [kbench --only list]'
set -e
ONLY=${1:-conv16_fwd,conv16_dgrad_mask,conv1x16_fwd}
for k in 1 2; do
 for v in head new; do cp _C_$v.so ncnet_amd/_C.so; echo "== $v"; timeout -k 10 100 python -u scripts/kbench.py --reps 20 --only $ONLY 2>&1 | grep -v amdgpu; done
done
