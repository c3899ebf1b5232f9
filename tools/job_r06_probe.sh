export YCX_ROUND=r06
O=gpurun_out/r06/j7; mkdir -p $O
# (1) isolated stem2 + a few convs, in-tree vs prescaled-SiLU probe lib
timeout -k 10 200 python -u tests/probes/stem2_bench.py > $O/stem2_B.txt 2>&1 || exit 1
YCX_LIB=$PWD/yolo-continuous_amd/ycx/libycx_A.so timeout -k 10 200 python -u tests/probes/stem2_bench.py > $O/stem2_A.txt 2>&1 || exit 1
tail -3 $O/stem2_B.txt; tail -3 $O/stem2_A.txt
# (2) concurrent bench A/B
bash tools/ab_bench.sh 2>&1 | tail -4
# (3) DVFS: tile 16 on two shapes, bf16 vs fp16, kernel cycles and time
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for DT in bf16 fp16; do
  CONV_DT=$DT CONV_SHAPES=0,14 timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES -d $R/$O/pmc_$DT -o run --output-format csv -- python3 $R/tests/probes/conv_bench.py 16 > $R/$O/pmc_$DT.log 2>&1 || { echo "pmc $DT failed"; tail -3 $R/$O/pmc_$DT.log; exit 1; }
  python3 - $R/$O/pmc_$DT $DT <<'PY'
import csv, glob, sys, collections
d, dt = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'conv' not in r['Kernel_Name']: continue
        agg[r['Grid_Size']][r['Counter_Name']].append(float(r['Counter_Value']))
for g, c in agg.items():
    print(dt, 'grid', g, {k: round(sum(v) / len(v)) for k, v in c.items()})
PY
  CONV_DT=$DT CONV_SHAPES=0,14 timeout -k 10 60 python3 $R/tests/probes/conv_bench.py 16 | tail -2
done
