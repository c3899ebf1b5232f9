#!/bin/bash
# Round-2 side configurations (run through gpurun): one bench line each into gpurun_out/r02/side_*.json.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02
run() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python bench.py --cpu-seconds 0 "$@" > gpurun_out/r02/side_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/r02/side_$n.log; return 1; }
  tail -1 gpurun_out/r02/side_$n.log > gpurun_out/r02/side_$n.json
  python -c "import json; d=json.load(open('gpurun_out/r02/side_$n.json')); print('$n', d['value'], d['ms_per_step'], d['p50_ms'], d['roofline']['kernel'], d['roofline']['frac'])"
}
run fp8_b64 --precision fp8 --batch 64 && run c4_1280 --size 1280 --batch 8 && run pipelined --mode pipelined && run dist --dist && run b64 --batch 64
