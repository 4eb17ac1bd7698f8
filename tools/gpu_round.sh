#!/bin/bash
# The one GPU-session driver: `gpurun -- bash tools/gpu_round.sh <target> [<target> ...]`.
# Every step runs under its own time limit; a test failure (exit 1) does not stop the session,
# a crash / abort / timeout does. Logs land in gpurun_out/<step>.log.
#   tests:    gputests kern eng batch tp tp8 rccl p2pu qkvsk bmmt t16t samp opsgpu smoke
#   benches:  bench bench20 serial benchtp2 benchdp2 bstep decode decode70 mixtral
#   profiles: stepprof decprof prefprof bmmpmc t16pmc blocks attntl bmmtl p2plat
#   A/B:      abold (the tree vs ab_old/, alternating), abprof (kernel tables, tree vs ab_old/)
#   final:    every GPU test + smoke + headline bench + step / decode kernel traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
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
PYT="python -u -m pytest -x -v --timeout-method thread -p no:cacheprovider"
prof() {  # prof <name> <timeout> <python args...>: rocprofv3 kernel trace + per-kernel summary
  local name=$1 to=$2; shift 2
  step "$name" "$to" rocprofv3 --kernel-trace --stats -d "gpurun_out/$name" -o k --output-format csv -- python3 "$@"
}
pmc() {  # pmc <name> <python args...>: one counter pass per run (8 SQ / 4 TCC / 2 GRBM slots)
  local name=$1; shift
  step "${name}A" 90 timeout -s KILL 80 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT -d "gpurun_out/${name}A" -o pmc --output-format csv -- python3 "$@"
  step "${name}B" 90 timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES \
    SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_RD -d "gpurun_out/${name}B" -o pmc --output-format csv -- python3 "$@"
  python3 tools/pmc_summary.py "gpurun_out/${name}A" "gpurun_out/${name}B" > "gpurun_out/${name}_summary.json" || true
}
for s in "$@"; do
  case $s in
    # ---- tests
    gputests) step gputests 1000 $PYT tests -m gpu --timeout 420 ;;
    kern) step kern 900 $PYT tests/test_kernels_gpu.py --timeout 120 ;;
    eng) step eng 900 $PYT tests/test_engine_gpu.py --timeout 300 ;;
    batch) step batch 600 $PYT tests/test_batch_gpu.py tests/test_batch_serving_gpu.py --timeout 300 ;;
    tp) step tp 900 $PYT tests/test_p2p_allreduce.py tests/test_tp_gpu.py --timeout 600 ;;
    tp8) step tp8 170 $PYT tests/test_tp8_gpu.py --timeout 160 -s ;;
    rccl) step rccl 400 $PYT tests/test_rccl_gpu.py tests/test_serve_tp_gpu.py --timeout 300 ;;
    p2pu) step p2pu 200 $PYT tests/test_p2p_allreduce.py --timeout 150 ;;
    tpepi) step tpepi 300 $PYT tests/test_tp_epilogue_gpu.py --timeout 120 ;;
    tpfault) step tpfault 700 $PYT tests/test_tp_fault_gpu.py --timeout 320 ;;
    qkvsk) step qkvsk 300 $PYT tests/test_kernels_gpu.py -k "qkv_splitk or attn_decode or bmm_rows" --timeout 120 ;;
    bmmt) step bmmt 400 $PYT tests/test_kernels_gpu.py -k "bmm or bprep" --timeout 120 ;;
    t16t) step t16t 400 $PYT tests/test_kernels_gpu.py -k "t16 or rmsnorm_f16 or attn_prefill" --timeout 120 ;;
    samp) step samp 300 $PYT tests/test_kernels_gpu.py -k sampler --timeout 120 ;;
    opsgpu) step opsgpu 600 $PYT tests/test_ops_gpu.py --timeout 120 ;;
    smoke) step smoke 300 python __graft_entry__.py smoke ;;
    # ---- benches
    bench) step bench 900 python bench.py --steps 3 --warmup 1 ;;
    bench20) step bench20 900 python bench.py --steps 20 --warmup 2 ;;
    serial) step serial 900 python bench.py --steps 10 --warmup 1 --clients 1 --max-batch 1 ;;
    benchtp2) step benchtp2 900 env LFK_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --parallel tp --steps 6 --warmup 1 ;;
    benchdp2) step benchdp2 900 env LFK_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --parallel dp --steps 4 --warmup 1 ;;
    bstep) step bstep 300 python tools/batch_bench.py --batches 1,6,8 --steps 48 ;;
    decode) step decode 600 python tools/decode_bench.py --gen 400 ;;
    decode70) step gen70 900 python tools/gen_model.py llama3-70b-q4_k_m
              step decode70 900 python tools/decode_bench.py --model llama3-70b-q4_k_m --steps 64 ;;
    mixtral) step genmx 900 python tools/gen_model.py mixtral-8x7b-q4_k_m
             step mixdec 600 python tools/decode_bench.py --model mixtral-8x7b-q4_k_m --steps 64
             step mixtral 900 python bench.py --model mixtral-8x7b-q4_k_m --steps 2 --warmup 1 ;;
    mixprof) export TMPDIR=/tmp; step genmx 900 python tools/gen_model.py mixtral-8x7b-q4_k_m
             prof mixprof 300 tools/decode_bench.py --model mixtral-8x7b-q4_k_m --steps 32 --no-graph
             python3 tools/prof_summary.py gpurun_out/mixprof/k_kernel_stats.csv > gpurun_out/mixprof_summary.md
             python3 tools/kernel_by_pred.py gpurun_out/mixprof/k_kernel_trace.csv > gpurun_out/mixprof_by_pred.md
             prof mixbprof 300 tools/batch_bench.py --model mixtral-8x7b-q4_k_m --batches 6 --steps 16
             python3 tools/step_kernels.py gpurun_out/mixbprof/k_kernel_trace.csv > gpurun_out/mixbprof_kernels.txt ;;
    tp8bench70) step gen70 900 python tools/gen_model.py llama3-70b-q4_k_m
                step tp8bench70 1100 env LFK_BENCH_DEVICE=0 GPU_MAX_HW_QUEUES=1 python -m torch.distributed.run --nnodes=1 \
                  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 8 --parallel tp \
                  --model llama3-70b-q4_k_m --steps 1 --warmup 0 --serial-steps 1 --clients ${TP8_CLIENTS:-6} ;;
    # ---- profiles
    stepprof) prof stepprof 300 tools/batch_bench.py --batches 6 --steps 32
              python3 tools/step_kernels.py gpurun_out/stepprof/k_kernel_trace.csv > gpurun_out/stepprof_kernels.txt
              python3 tools/step_slots.py gpurun_out/stepprof/k_kernel_trace.csv >> gpurun_out/stepprof_kernels.txt ;;
    dec70prof) step gen70 900 python tools/gen_model.py llama3-70b-q4_k_m
               prof dec70prof 400 tools/decode_bench.py --model llama3-70b-q4_k_m --steps 16 --no-graph
               python3 tools/prof_summary.py gpurun_out/dec70prof/k_kernel_stats.csv > gpurun_out/dec70prof_summary.md
               python3 tools/kernel_by_pred.py gpurun_out/dec70prof/k_kernel_trace.csv > gpurun_out/dec70prof_by_pred.md ;;
    decprof) prof decprof 300 tools/decode_bench.py --steps 64 --no-graph
             python3 tools/prof_summary.py gpurun_out/decprof/k_kernel_stats.csv > gpurun_out/decprof_summary.md ;;
    prefprof) prof prefprof 300 tools/decode_bench.py --prompt 512 --steps 8 --slots 2 ;;
    # the bench's admission prefill (7-slot engine): 387-token prompts alone, then 6 jointly
    admprof) prof admprof 300 tools/prefill_bench.py --T 387 --reps 4 --joint 6
             python3 tools/kernel_by_pred.py gpurun_out/admprof/k_kernel_trace.csv --min-calls 4 --grid > gpurun_out/admprof_by_pred.md ;;
    bmmpmc) pmc bmmpmc tools/batch_bench.py --batches 6 --steps 4 ;;
    t16pmc) pmc t16pmc tools/gemm_bench.py --eager --reps 5 --T 512 --t16 ;;
    # the wave-owned projections by part (full / weights + MFMA / weights only), counters per kernel
    wtpmc) pmc wtpmc tools/boundary_bench.py --debug 0,6,4 --chains gu,down --n 12 --norm ;;
    blocks) step blocks 200 python tools/step_blocks.py --json gpurun_out/blocks.json ;;
    attntl) step attntl 200 python tools/attn_timeline.py --rows 6 --L 700 ;;
    bmmtl) step bmmtl 200 python tools/bmm_timeline.py --rows 6 --json gpurun_out/bmm_tl6.json ;;
    gemmt) step gemmt 400 bash -c 'for T in 384 512 1024 2304; do python tools/gemm_bench.py --T $T --t16 || exit 1; done' ;;
    bound) step bound 200 python tools/boundary_bench.py --json gpurun_out/bound_default.json
           step bound_devka 200 env HIP_FORCE_DEV_KERNARG=1 python tools/boundary_bench.py --json gpurun_out/bound_devka1.json
           step bound_hostka 200 env HIP_FORCE_DEV_KERNARG=0 python tools/boundary_bench.py --json gpurun_out/bound_devka0.json ;;
    p2plat) step p2plat 300 python tools/p2p_latency.py --ranks 2,4,8 --json gpurun_out/p2p_latency.json ;;
    # ---- same-box A/B against the older build staged in ab_old/ (drop ./ab_old from .gpurunignore)
    abold) for r in 1 2; do
             step "abo_new_$r" 200 python tools/batch_bench.py --batches 1,6,8
             step "abo_old_$r" 200 python ab_old/tools/batch_bench.py --batches 1,6,8
           done ;;
    abprof) for v in new old; do
              bb=tools/batch_bench.py; [ $v = old ] && bb=ab_old/tools/batch_bench.py
              prof "abp_$v" 240 $bb --batches 6 --steps 32
              python3 tools/step_kernels.py "gpurun_out/abp_$v/k_kernel_trace.csv" > "gpurun_out/abp_$v.txt"
              python3 tools/step_slots.py "gpurun_out/abp_$v/k_kernel_trace.csv" >> "gpurun_out/abp_$v.txt"
            done ;;
    # ---- same-box A/B of an env switch of the tree's build: AB_ENV="LFK_X=0" (alternating runs,
    #      then a kernel table of each)
    abenv) for r in 1 2; do
             step "abe_on_$r" 200 python tools/batch_bench.py --batches 1,6,8 --steps 64
             step "abe_off_$r" 200 env $AB_ENV python tools/batch_bench.py --batches 1,6,8 --steps 64
           done
           prof abe_on_prof 240 tools/batch_bench.py --batches 6 --steps 32
           python3 tools/step_slots.py gpurun_out/abe_on_prof/k_kernel_trace.csv > gpurun_out/abe_on_slots.txt
           step abe_off_prof 240 env $AB_ENV rocprofv3 --kernel-trace --stats -d gpurun_out/abe_off_prof -o k \
             --output-format csv -- python3 tools/batch_bench.py --batches 6 --steps 32
           python3 tools/step_slots.py gpurun_out/abe_off_prof/k_kernel_trace.csv > gpurun_out/abe_off_slots.txt ;;
    # ---- same-box A/B of several env configurations: AB_CONFIGS="A=1,B=2 C=3" (space-separated
    #      configs, comma-separated vars; "-" = the defaults), alternating, two rounds
    abmulti) for r in 1 2; do
               i=0
               for c in $AB_CONFIGS; do
                 i=$((i + 1))
                 step "abm_${i}_$r" 200 env $(echo "$c" | tr ',' ' ' | sed 's/^-$//') python tools/batch_bench.py --batches 6,8 --steps 64
               done
             done ;;
    # ---- round-end check of the committed tree
    final) bash "$0" gputests smoke bench20 serial stepprof decprof || exit $? ;;
    *) echo "unknown target $s" >&2; exit 2 ;;
  esac
done
