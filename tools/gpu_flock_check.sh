set -u
mkdir -p gpurun_out/flock
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graph.py -m gpu -p no:cacheprovider > gpurun_out/flock/pytest_graph.log 2>&1; rc=$?; tail -15 gpurun_out/flock/pytest_graph.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --scenario flocking --n-agents 8 --substeps 0 --steps 50 --warmup 10 --cpu-steps 0 > gpurun_out/flock/c5.json 2> gpurun_out/flock/c5.log; rc=$?; cat gpurun_out/flock/c5.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --scenario flocking --n-agents 8 --substeps 0 --steps 50 --warmup 10 --cpu-steps 0 --graph off > gpurun_out/flock/c5_eager.json 2>> gpurun_out/flock/c5.log; cat gpurun_out/flock/c5_eager.json
