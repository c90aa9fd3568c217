# Round deliverables on the GPU box for the current tree (run via gpurun):
#   gpurun --timeout 1200 -- 'bash tools/gpu_round.sh r04_v1 [quick]'
# Full GPU parity, bench C2 with CPU baseline, C1/C3/C4/cerberus bench lines, the
# emulated 8-way shards (C2 at 2/4/8 replicated, C2/C3 partitioned and C3
# replicated at 8), kernel-trace stats, PMC FETCH/WRITE passes + counter
# calibration, the tile pass's traffic by request class (tools/pmc_classes.sh,
# needs zenith_amd/variants/dbg built).  "quick" stops after the bench lines.
# Every GPU step has its own time limit; the first failure ends the run.
set -o pipefail
export TMPDIR=/tmp
V=${1:?version tag}
O=gpurun_out/$V
mkdir -p $O
if [ "$2" != pmc ]; then  # "pmc": the profiler passes only
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench.err || exit 2
for c in c1 c3 c4 cerberus c2x c3x; do timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2>> $O/bench.err || exit 3; done
for g in 2 4 8; do timeout -k 10 200 python bench.py --emulate-shard $g --no-cpu-baseline > $O/bench_c2_shard$g.json 2>> $O/bench.err || exit 3; done
for c in c2 c3; do timeout -k 10 200 python bench.py --config $c --emulate-shard 8 --setup partitioned --no-cpu-baseline > $O/bench_${c}_shard8_part.json 2>> $O/bench.err || exit 3; done
timeout -k 10 200 python bench.py --config c3 --emulate-shard 8 --no-cpu-baseline > $O/bench_c3_shard8.json 2>> $O/bench.err || exit 3
[ "$2" = quick ] && { echo done; exit 0; }
fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --cold-copies 0 --no-census > $O/kt.log 2>&1 || exit 4
python3 tools/kt_summary.py $O/kt/run_kernel_stats.csv --config c2 -o $O/kt_c2.json > /dev/null || exit 4
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o run --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline --cold-copies 0 --no-census > $O/pf.log 2>&1 || exit 5
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o run --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline --cold-copies 0 --no-census > $O/pw.log 2>&1 || exit 6
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $O/cf -o run --output-format csv -- tools/build/pmc_calib > $O/calib_known.txt 2>&1 || exit 7
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $O/cw -o run --output-format csv -- tools/build/pmc_calib > $O/calib_w.txt 2>&1 || exit 8
bash tools/pmc_classes.sh $V || exit 9
C=gpurun_out/pmcc_$V
python3 tools/pmc_summary.py --fetch $O/pf/run_counter_collection.csv --write $O/pw/run_counter_collection.csv \
  --calib $O/cf/run_counter_collection.csv $O/cw/run_counter_collection.csv --calib-known $O/calib_known.txt \
  --config c2 --classes $C/dbg0/run_counter_collection.csv $C/ids/run_counter_collection.csv \
  $C/attrs/run_counter_collection.csv $C/recs/run_counter_collection.csv $C/noraster/run_counter_collection.csv \
  -o $O/pmc_c2.json > /dev/null || exit 10
echo done
