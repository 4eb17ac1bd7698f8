#!/bin/bash
# One GPU session: kernel numerics, engine tests, smoke, raw decode timing.
# Test failures (exit 1) do not stop the session; a crash/abort/timeout does.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name" >&2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >&2
  tail -5 "gpurun_out/$name.log" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc" >&2; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    kern) step kern 900 python -m pytest tests/test_kernels_gpu.py -q -p no:cacheprovider ;;
    eng) step eng 900 python -m pytest tests/test_engine_gpu.py -q -p no:cacheprovider ;;
    gputests) step gputests 1200 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    smoke) step smoke 300 python __graft_entry__.py smoke ;;
    decode) step decode 600 python tools/decode_bench.py --gen 400 ;;
    micro) step micro 300 python tools/launch_microbench.py ;;
    gemvb) step gemvb 300 python tools/gemv_bench.py --debug ;;
    sweep) step sweep 900 bash tools/gemv_sweep.sh ;;
    timeline) step timeline 300 python tools/gemv_timeline.py ;;
    sampb) step sampb 300 python tools/sampler_bench.py ;;
    variants) step variants 900 bash tools/gemv_variants.sh ;;
    profgemv) export TMPDIR=/tmp; step profgemv 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profgemv -o gemv \
            --output-format csv -- python3 tools/gemv_bench.py --eager --reps 20 ;;
    pdtest) step pdtest 400 python -u -m pytest tests/test_pdecode_gpu.py -v --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    pddebug) step pddebug 300 python -u tools/pdecode_debug.py ;;
    pddebug4) step pddebug4 300 python -u tools/pdecode_debug.py --spec pd-llama-g4 --n 100 ;;
    pdtl) step pdtl 300 python -u tools/pdecode_timeline.py ;;
    pdtl1) LFK_PDECODE_DBG=1 step pdtl1 300 python -u tools/pdecode_timeline.py ;;
    pdtl2) LFK_PDECODE_DBG=2 step pdtl2 300 python -u tools/pdecode_timeline.py ;;
    pdtl3) LFK_PDECODE_DBG=3 step pdtl3 300 python -u tools/pdecode_timeline.py ;;
    pdacct) step pdacct 300 python -u tools/pdecode_acct.py ;;
    pdacct2) LFK_PDECODE_DBG=2 step pdacct2 300 python -u tools/pdecode_acct.py ;;
    pditem) step pditem 120 python -u tools/pd_item_bench.py ;;
    gvpmc) export TMPDIR=/tmp; step gvpmc 90 timeout -s KILL 80 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d gpurun_out/gvpmc -o pmc --output-format csv -- python3 tools/gemv_bench.py --eager --reps 20 --only q4k ;;
    pdcheck) step pdcheck 300 python -u tools/pdecode_check.py ;;
    pdcheck70) step pdcheck70 600 python -u tools/pdecode_check.py --model llama3-70b-q4_k_m --steps 16 ;;
    pdpmc1) export TMPDIR=/tmp; step pdpmc1 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES -d gpurun_out/pdpmc1 -o pmc --output-format csv -- python3 tools/pdecode_prof.py --steps 4 ;;
    pdpmc2) export TMPDIR=/tmp; step pdpmc2 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INST_CYCLES_SALU -d gpurun_out/pdpmc2 -o pmc --output-format csv -- python3 tools/pdecode_prof.py --steps 4 ;;
    opsgpu) step opsgpu 600 python -m pytest tests/test_ops_gpu.py -q -p no:cacheprovider ;;
    bench) step bench 900 python bench.py --steps 3 --warmup 1 ;;
    prof) export TMPDIR=/tmp; step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o decode \
            --output-format csv -- python3 tools/decode_bench.py --steps 64 --no-graph ;;
  esac
done
