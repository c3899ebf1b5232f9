# tile 16 / 18 build variants (VARS: lib suffixes), isolated, interleaved
mkdir -p gpurun_out/r06
O=gpurun_out/r06/stagger.txt; : > $O
for r in 1 2; do
  for v in ${VARS:-hip SP NP}; do
    echo "== $v" >> $O
    YCX_LIB=$PWD/yolo-continuous_amd/ycx/libycx_$v.so CONV_SHAPES=0,5,14,16,21,26,12 timeout -k 10 120 python -u tests/probes/conv_bench.py 16 18 >> $O 2>&1 || exit 1
  done
done
python - <<'PY'
import re, collections
cur=None; d=collections.defaultdict(lambda: collections.defaultdict(list))
for line in open('gpurun_out/r06/stagger.txt'):
    m=re.match(r'== (\S+)', line)
    if m: cur=m.group(1); continue
    m=re.match(r'(\(.*?\))\s+(.*)', line)
    if not m: continue
    for t, ms in re.findall(r't(\d+): ([\d.]+) ms', m.group(2)):
        d[(m.group(1), t)][cur].append(float(ms)*1000)
for k, v in d.items():
    print(k, ' '.join(f"{lib}={min(x):.1f}" for lib, x in v.items()))
PY
