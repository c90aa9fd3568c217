set -o pipefail
O=gpurun_out/dist3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "rccl" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --no-cpu-baseline --force-dist > $O/c2_dist1.json 2>>$O/err || exit 2
ZR_RCCL_NO_ALLTOALL=1 timeout -k 10 120 python bench.py --no-cpu-baseline --force-dist > $O/c2_dist1_p2p.json 2>>$O/err || exit 3
timeout -k 10 120 python bench.py --no-cpu-baseline --force-dist --setup replicated > $O/c2_dist1_rep.json 2>>$O/err || exit 4
timeout -k 10 120 python bench.py --no-cpu-baseline > $O/c2.json 2>>$O/err || exit 5
echo done
