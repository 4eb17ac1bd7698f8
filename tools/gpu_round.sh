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
    rccl) step rccl 400 python -u -m pytest tests/test_rccl_gpu.py tests/test_serve_tp_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    p2pu) step p2pu 200 env LFK_P2P_UNCACHED=1 python -u -m pytest tests/test_p2p_allreduce.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider ;;
    tp) step tp 460 python -u -m pytest tests/test_p2p_allreduce.py tests/test_tp_gpu.py -x -v --timeout 420 --timeout-method thread -p no:cacheprovider ;;
    bmmt) step bmmt 400 python -u -m pytest tests/test_kernels_gpu.py -k "bmm or bprep" -q --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    bmmtl) step bmmtl 200 python tools/bmm_timeline.py --rows 6 --json gpurun_out/bmm_tl6.json ;;
    attntl) step attntl 200 python tools/attn_timeline.py --rows 6 --L 700 ;;
    attntl1) step attntl1 200 python tools/attn_timeline.py --rows 1 --L 700 ;;
    bstep) step bstep 300 python tools/batch_bench.py --batches 1,6,8 --steps 48 ;;
    qkvsk) step qkvsk 300 python -u -m pytest tests/test_kernels_gpu.py -k "qkv_splitk or attn_decode or bmm_rows" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    absk) step absk0 200 env LFK_QKV_SK=0 python tools/batch_bench.py --batches 6,8 --steps 64
          step absk1 200 python tools/batch_bench.py --batches 6,8 --steps 64
          step absk0b 200 env LFK_QKV_SK=0 python tools/batch_bench.py --batches 6,8 --steps 64
          step absk1b 200 python tools/batch_bench.py --batches 6,8 --steps 64 ;;
    blocks) step blocks1 200 python tools/step_blocks.py --json gpurun_out/blocks_sk1.json
            step blocks0 200 env LFK_QKV_SK=0 python tools/step_blocks.py --json gpurun_out/blocks_sk0.json ;;
    sksweep) for c in 8,8 4,6 4,8 2,3 16,6; do
               step "sk_$c" 200 env LFK_QKV_SK_PARTS=${c%,*} LFK_QKV_SK_TPG=${c#*,} python tools/batch_bench.py --batches 6 --steps 64
             done ;;
    xfirst) step xf_blocks1 200 env LFK_WT_XFIRST=1 LFK_QKV_SK_PARTS=4 python tools/step_blocks.py --json gpurun_out/blocks_xf1.json
            step xf_blocks0 200 env LFK_QKV_SK_PARTS=4 python tools/step_blocks.py --json gpurun_out/blocks_xf0.json
            for x in 0 1 0 1; do step "xf_bench_$x" 200 env LFK_WT_XFIRST=$x LFK_QKV_SK_PARTS=4 python tools/batch_bench.py --batches 6 --steps 64; done ;;
    p2pprobe) step p2pprobe0 120 python tools/p2p_probe.py
              step p2pprobe1 120 python tools/p2p_probe.py --junk ;;
    abold) step abold 600 bash tools/gpu_ab_old.sh ;;
    stepprof) export TMPDIR=/tmp; step stepprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sprof -o bstep --output-format csv -- python3 tools/batch_bench.py --batches 6 --steps 32
          python3 tools/step_kernels.py gpurun_out/sprof/bstep_kernel_trace.csv > gpurun_out/sprof_kernels.txt ;;
    samp) step samp 300 python -u -m pytest tests/test_kernels_gpu.py -k sampler -v --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    kern) step kern 900 python -m pytest tests/test_kernels_gpu.py -q -p no:cacheprovider ;;
    eng) step eng 900 python -m pytest tests/test_engine_gpu.py -q -p no:cacheprovider ;;
    gputests) step gputests 1000 python -u -m pytest tests -m gpu -q --timeout 420 --timeout-method thread -p no:cacheprovider ;;
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
    gvpmc) export TMPDIR=/tmp; step gvpmc 90 timeout -s KILL 80 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d gpurun_out/gvpmc -o pmc --output-format csv -- python3 tools/gemv_bench.py --eager --reps 20 --only q4k ;;
    opsgpu) step opsgpu 600 python -m pytest tests/test_ops_gpu.py -q -p no:cacheprovider ;;
    gemmb) step gemmb 300 bash -c 'python tools/gemm_bench.py --T 512 && python tools/gemm_bench.py --T 2048' ;;
    gemmt) step gemmt 300 bash -c 'for T in 384 512 2048 2304; do python tools/gemm_bench.py --T $T && python tools/gemm_bench.py --T $T --t16 || exit 1; done; for c in 8,128 8,64 4,64; do LFK_T16_CFG=$c python tools/gemm_bench.py --T 512 --t16 || exit 1; done' ;;
    gemmt2) step gemmt2 300 bash -c 'for T in 2304 2400 1536; do python tools/gemm_bench.py --T $T --t16 && LFK_T16_CFG=8,128 python tools/gemm_bench.py --T $T --t16 || exit 1; done' ;;
    gemmt4) step gemmt4 300 bash -c 'for T in 384 512 1024 2304; do python tools/gemm_bench.py --T $T --t16 || exit 1; done' ;;
    gemmt3) step gemmt3 400 bash -c 'for T in 384 1024 1536 2304; do for c in 8,128 8,64 4,64; do echo cfg=$c; LFK_T16_CFG=$c python tools/gemm_bench.py --T $T --t16 || exit 1; done; done' ;;
    t16t) step t16t 400 python -u -m pytest tests/test_kernels_gpu.py -k "t16 or rmsnorm_f16 or attn_prefill" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    gemmpmc) export TMPDIR=/tmp; step gemmpmcA 90 timeout -s KILL 80 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT \
            -d gpurun_out/gemmpmcA -o pmc --output-format csv -- python3 tools/gemm_bench.py --eager --reps 5 --only gateup
            step gemmpmcB 90 timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
            -d gpurun_out/gemmpmcB -o pmc --output-format csv -- python3 tools/gemm_bench.py --eager --reps 5 --only gateup ;;
    t16pmc) export TMPDIR=/tmp; step t16pmcA 90 timeout -s KILL 80 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT \
            -d gpurun_out/t16pmcA -o pmc --output-format csv -- python3 tools/gemm_bench.py --eager --reps 5 --T 512 --t16
            step t16pmcB 90 timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
            -d gpurun_out/t16pmcB -o pmc --output-format csv -- python3 tools/gemm_bench.py --eager --reps 5 --T 512 --t16
            step prefprof 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prefprof -o pre --output-format csv -- python3 tools/decode_bench.py --prompt 512 --steps 8 --slots 2 ;;
    bench) step bench 900 python bench.py --steps 3 --warmup 1 ;;
    bench20) step bench20 900 python bench.py --steps 20 --warmup 2 ;;
    benchtp2) LFK_BENCH_DEVICE=0 step benchtp2 900 python bench.py --gpus 2 --steps 12 --warmup 2 ;;
    benchdp2) LFK_BENCH_DEVICE=0 step benchdp2 900 python bench.py --gpus 2 --parallel dp --steps 12 --warmup 2 ;;
    batch) step batch 600 python -u -m pytest tests/test_batch_gpu.py tests/test_batch_serving_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    prof) export TMPDIR=/tmp; step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o decode \
            --output-format csv -- python3 tools/decode_bench.py --steps 64 --no-graph ;;
  esac
done
