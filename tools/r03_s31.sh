# per-kernel times of the NMS chain at C2 (bench load, tests/probes/nms_phases.py, under rocprof): HEAD (base) vs split prep (hip)
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03/pm
cd /tmp && export TMPDIR=/tmp
for v in base hip; do
YCX_LIB=$R/yolo-continuous_amd/ycx/libycx_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03/pm/$v -o run --output-format csv -- python3 $R/tests/probes/nms_phases.py > $R/gpurun_out/r03/pm/$v.log 2>&1 || { tail -5 $R/gpurun_out/r03/pm/$v.log; exit 1; }
echo "== $v"; python3 - $R/gpurun_out/r03/pm/$v/run_kernel_stats.csv <<'PY'
import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r:-float(r['TotalDurationNs']))[:10]:
    print(f"calls {r['Calls']:>6} avg {float(r['AverageNs'])/1000:8.1f}us  {r['Name'][:70]}")
PY
done
