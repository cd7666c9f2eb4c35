set -o pipefail
O=gpurun_out/v6; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q --timeout 200 --timeout-method thread -k "graph or overlap" > $O/pytest.log 2>&1 || { echo TEST FAILED; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do timeout -k 10 400 python tools/overlap_ab.py "3,3,1" "3,2,1" "3,4,1" "2,3,1" "1,0,1" -- --steps 60 >> $O/ab.txt 2>&1 || { echo AB FAILED; cat $O/ab.txt; exit 1; }; done
cat $O/ab.txt
# more hardware queues per process (HIP's default is 4): two / three batches in flight
for q in 8; do
  for nf in 2 3; do
    echo "GPU_MAX_HW_QUEUES=$q inflight $nf" >> $O/ab_q.txt
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python tools/overlap_ab.py "3,3,1" "0" -- --steps 60 --inflight $nf >> $O/ab_q.txt 2>&1 || { echo AB FAILED; cat $O/ab_q.txt; exit 1; }
  done
done
cat $O/ab_q.txt
