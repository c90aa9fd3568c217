set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1
for v in 0 8 16 1; do ZR_DEBUG=$v timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/bench5_d$v.json 2>>gpurun_out/bench5.err || exit 1; done
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc1 -o run --output-format csv -- $B > gpurun_out/pmc1.log 2>&1 || exit 2
timeout -k 10 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc2 -o run --output-format csv -- $B > gpurun_out/pmc2.log 2>&1 || exit 3
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc3 -o run --output-format csv -- $B > gpurun_out/pmc3.log 2>&1 || exit 4
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc4 -o run --output-format csv -- $B > gpurun_out/pmc4.log 2>&1 || exit 5
for f in gpurun_out/bench5_d*.json; do echo $f; python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items()})" $f; done
