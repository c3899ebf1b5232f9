# sparse (trained-weights-like) and dense post micro-bench: HEAD vs split bucketing, alternating
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2; do for v in base hip; do for sh in -3 0; do
echo -n "$v shift $sh: "; YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_$v.so timeout -k 10 120 python bench.py --post-micro --obj-shift $sh 2>&1 | grep -v amdgpu | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done; done; done
