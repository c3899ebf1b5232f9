cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r06cp
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-seconds 0 --fp16-steps 0 --pipelined-steps 0 --image-in-steps 0 --latency-steps 0 --roofline-steps 1 --steps 50 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
f=$(find $O/p -name '*kernel_stats.csv' | head -n 1); cp $f $O/stats.csv
t=$(find $O/p -name '*kernel_trace.csv' | head -n 1); python3 - "$t" <<'P'
import csv,sys,collections
rows=list(csv.DictReader(open(sys.argv[1])))
cp=[r for r in rows if 'copyBuffer' in r['Kernel_Name']]
print(len(rows), len(cp))
c=collections.Counter((r.get('Grid_Size_X') or r.get('Grid_Size'), r.get('Workgroup_Size_X') or r.get('Workgroup_Size')) for r in cp)
print(c.most_common(10))
print(list(rows[0].keys()))
P
rm -rf $O/p
