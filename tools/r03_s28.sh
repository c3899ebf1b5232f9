# end-of-round profile: rocprof stats + PMC traffic + bench (profile_round), then the side configs' bench lines
R=$GRAFT_REPO_ROOT
cd $R
bash tools/profile_round.sh r03 || exit 1
for cfg in "fp8_b64:--precision fp8 --batch 64" "b64:--batch 64" "c4_1280:--size 1280 --batch 8" "fp16:--precision fp16"; do
name=${cfg%%:*}; args=${cfg#*:}
timeout -k 10 300 python bench.py --cpu-seconds 0 $args > gpurun_out/r03/side_$name.log 2>&1 || { tail -5 gpurun_out/r03/side_$name.log; exit 1; }
tail -1 gpurun_out/r03/side_$name.log > gpurun_out/r03/side_$name.json
echo -n "$name "; python -c "import json; d=json.load(open('gpurun_out/r03/side_$name.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
done
