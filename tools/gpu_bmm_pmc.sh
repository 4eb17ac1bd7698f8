# bmm counters: microbenchmark (full math vs weight stream only), then PMC passes over the
# B=6 batch step, each pass its own run (counter slots: 8 SQ, 4 TCC, 2 GRBM).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/bmm_bench.py --rows 1,6,8 > gpurun_out/bmmb_full.json 2>&1 || exit 1
timeout -k 10 120 python tools/bmm_bench.py --rows 1,6,8 --debug 1 > gpurun_out/bmmb_stream.json 2>&1 || exit 1
cat gpurun_out/bmmb_full.json gpurun_out/bmmb_stream.json
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT \
  -d gpurun_out/pmcA -o pmc --output-format csv -- python3 tools/batch_bench.py --batches 6 --steps 4 > gpurun_out/pmcA.log 2>&1 || { tail -5 gpurun_out/pmcA.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM \
  -d gpurun_out/pmcB -o pmc --output-format csv -- python3 tools/batch_bench.py --batches 6 --steps 4 > gpurun_out/pmcB.log 2>&1 || { tail -5 gpurun_out/pmcB.log; exit 1; }
echo done
