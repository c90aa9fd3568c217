# Cold-cache (HBM-honest) bench lines: geometry copies cycled frame to frame so the
# input footprint exceeds the 256 MiB Infinity Cache, plus a
# kernel-trace of the C2 rotated run.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-rot}; mkdir -p $O
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/c2_rot1.json 2>>$O/err || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --rotate 3 > $O/c2_rot3.json 2>>$O/err || exit 2
timeout -k 10 200 python bench.py --no-cpu-baseline --config c3 --rotate 2 > $O/c3_rot2.json 2>>$O/err || exit 3
timeout -k 10 200 python bench.py --no-cpu-baseline --config c1 --rotate 32 > $O/c1_rot32.json 2>>$O/err || exit 4
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --rotate 3 > $O/kt.log 2>&1 || exit 5
echo done
