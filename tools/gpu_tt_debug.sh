set -u
mkdir -p gpurun_out
DCT_GRAPH=0 timeout -k 10 300 python -X faulthandler bench.py --model tabtransformer --steps 10 --warmup 5 --rows 1000000 > gpurun_out/tt_nograph.log 2>&1; echo "nograph rc=$?"
tail -30 gpurun_out/tt_nograph.log | cut -c1-600
timeout -k 10 300 python -X faulthandler bench.py --model tabtransformer --steps 10 --warmup 5 --rows 1000000 > gpurun_out/tt_graph.log 2>&1; echo "graph rc=$?"
tail -40 gpurun_out/tt_graph.log | cut -c1-600
