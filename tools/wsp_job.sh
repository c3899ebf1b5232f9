# tile 57 (warp-specialised) parity + isolated timing against tile 16 (development job, via gpurun)
export YCX_ROUND=r06
O=gpurun_out/r06/wsp; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "wsp or (bf16_tiles and 57)" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tests/probes/conv_bench.py 16 57 > $O/bench_16_57.txt 2>&1 || exit 1
for v in ${WSP_VARIANTS:-P2 P3 P33}; do
  YCX_LIB=$PWD/yolo-continuous_amd/ycx/libycx_$v.so timeout -k 10 300 python -u tests/probes/conv_bench.py 57 > $O/bench_57_$v.txt 2>&1 || exit 1
done
python - <<'PY'
import glob, re
rows = {}
for f in sorted(glob.glob('gpurun_out/r06/wsp/bench_*.txt')):
    tag = f.split('bench_')[1][:-4]
    for line in open(f):
        m = re.match(r'(\(.*?\))\s+(.*)', line)
        if not m: continue
        for t, ms in re.findall(r't(\d+): ([\d.]+) ms', m.group(2)):
            rows.setdefault(m.group(1), {})[f"{tag}:t{t}"] = float(ms) * 1000
for sh, d in rows.items():
    print(sh, ' '.join(f"{k}={v:.1f}" for k, v in d.items()))
PY
# SQ counters of one launch shape (40^2 256->256 3x3, bs 32) for tile 16 and tile 57
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for T in 16 57; do
  CONV_SHAPES=0 timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $R/$O/pmc_$T -o run --output-format csv -- python3 $R/tests/probes/conv_bench.py $T > $R/$O/pmc_$T.log 2>&1 || { echo "pmc $T failed"; tail -5 $R/$O/pmc_$T.log; exit 1; }
  python3 $R/tests/probes/pmc_summary.py $R/$O/pmc_$T conv > $R/$O/pmc_$T.txt; echo "== tile $T"; cat $R/$O/pmc_$T.txt
  rm -rf $R/$O/pmc_$T
done
