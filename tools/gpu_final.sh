# Round-end check of the tree as committed: every GPU test, smoke(), the headline bench, and a
# kernel trace of the B = 6 batch step (its stats CSV is copied into profiles/).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/final_tests.log 2>&1 || { tail -30 gpurun_out/final_tests.log; exit 1; }
tail -2 gpurun_out/final_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || exit 1
cat gpurun_out/final_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fprof -o bstep --output-format csv -- \
  python3 tools/batch_bench.py --batches 6 --steps 32 > gpurun_out/fprof.log 2>&1 || { tail -20 gpurun_out/fprof.log; exit 1; }
echo done
# single-row decode (the reference's serving mode): kernel stats of graph-free decode steps
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fdec -o dec --output-format csv -- \
  python3 tools/decode_bench.py --steps 64 --no-graph > gpurun_out/fdec.log 2>&1 || { tail -20 gpurun_out/fdec.log; exit 1; }
echo done2
