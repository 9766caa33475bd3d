#!/bin/bash
# Round-4 GPU call: a chosen list of named steps, each under its own time limit, stopping at the
# first failure.  usage: tools/gpu_r4.sh TAG step [step ...]
#   tests        all -m gpu tests            bench        bench.py default line
#   bench_trace  rocprofv3 stats of bench.py corr100k     rocprofv3 stats, C3 correlation (tau 0.5)
#   corr1m       rocprofv3 stats, 1M-pod correlation (tau 0.5)
#   ranking      tools/ranking_ablation_c4.py (C4 mesh, 2 seeds)
#   ppr          rocprofv3 stats of the C4 PageRank propagate   logs / tmpl  same for logs / templates
#   c5           tools/bench_stream.py (C5 window)
#   c5_phases    the same, the three parts one after another with per-part events
set -u
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
finish() {
  find $O -name '*.db' -delete
  find $O -name '*kernel_trace.csv' -size +4M -delete
}
trap finish EXIT
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?; echo "$name EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { echo "stop after $name"; tail -30 $O/$name.log; exit $rc; }
  tail -3 $O/$name.log
}
prof() {  # prof NAME SECONDS ARGS... (rocprofv3 kernel-trace stats of python3 ARGS)
  local name=$1 secs=$2; shift 2
  step $name $secs rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- python3 "$@"
}
pmc() {  # pmc NAME WHAT COUNTERS... (one counter pass of tools/prof_kernels.py WHAT, its own kill timeout)
  local name=$1 what=$2; shift 2
  step $name 120 timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o run -- python3 tools/prof_kernels.py $what --reps 1
}
for s in "$@"; do
  case $s in
    probe) step probe 60 tools/bin/buffer_range_probe ;;
    tests_new) step tests_new 600 python3 -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread -k "empty_rank or cold_solve_fresh or bench_gpus" ;;
    bench_n4) step bench_n4 700 env KRCA_BENCH_BACKEND=gloo python3 bench.py --gpus 4 --steps 3 --warmup 1 --no-corr --cpu-runs 2 --cpu-warmup 1 ;;
    bench_n2) step bench_n2 600 env KRCA_BENCH_BACKEND=gloo python3 bench.py --gpus 2 --steps 5 --warmup 2 ;;
    tests_logs) step tests_logs 600 python3 -u -m pytest tests -m gpu -x -v -rP --timeout 240 --timeout-method thread -k "log_scan or c2mini or c5 or stream or logs" ;;
    pprw_*) export KRCA_LIB=$PWD/kubernetes-rca-system_amd/lib/libkrca_${s#pprw_}.so; prof $s 300 tools/ppr_bench.py --reps 10; unset KRCA_LIB ;;
    pprbase) prof pprbase 300 tools/ppr_bench.py --reps 10 ;;
    pprx_*) o=${s#pprx_}; prof $s 300 tools/ppr_bench.py --order ${o%_*} --xcd ${o##*_} --check --reps 10 ;;
    logs_fused1) export KRCA_LOG_FUSED=1; prof logs_fused1 300 tools/prof_kernels.py logs --reps 5; unset KRCA_LOG_FUSED ;;
    logs_fused2) export KRCA_LOG_FUSED=2; prof logs_fused2 300 tools/prof_kernels.py logs --reps 5; unset KRCA_LOG_FUSED ;;
    log_timing0) export KRCA_LIB=$PWD/kubernetes-rca-system_amd/lib/libkrca_ltime.so; step log_timing0 300 python3 tools/log_timing.py; unset KRCA_LIB ;;
    log_timing2) export KRCA_LOG_FUSED=2 KRCA_LIB=$PWD/kubernetes-rca-system_amd/lib/libkrca_ltime.so; step log_timing2 300 python3 tools/log_timing.py; unset KRCA_LIB KRCA_LOG_FUSED ;;
    logs_unfused) export KRCA_LOG_FUSED=0; prof logs_unfused 300 tools/prof_kernels.py logs --reps 5; unset KRCA_LOG_FUSED ;;
    tests) step tests 900 python3 -u -m pytest tests -m gpu -x -v -rP --timeout 240 --timeout-method thread ;;
    tests_corrq) step tests_corrq 600 python3 -u -m pytest tests/test_gpu_corr.py -x -v -rP --timeout 240 --timeout-method thread -k "batches or c3_every or full_vs" ;;
    tests_corr) step tests_corr 600 python3 -u -m pytest tests/test_gpu_corr.py -x -v -rP --timeout 240 --timeout-method thread ;;
    bench) step bench 300 python3 bench.py ;;
    score_lds) step score_lds 300 python3 tools/score_ab.py --only pipe_c20,lds,lds_default_policy --rounds 3 --reps 5 ;;
    tests_score) step tests_score 300 python3 -u -m pytest tests/test_gpu_kernels.py -x -v -rP --timeout 120 --timeout-method thread -k "rolling_score" ;;
    benchnt_*) v=${s#benchnt_}; export KRCA_PPR_NT=${v%%_*}; step $s 300 python3 bench.py --no-corr --no-cpu-baseline --no-verify; unset KRCA_PPR_NT ;;
    benchx_*) v=${s#benchx_}; export KRCA_PPR_XCD=${v%%_*}; step $s 300 python3 bench.py --no-corr --no-cpu-baseline --no-verify --steps 20; unset KRCA_PPR_XCD ;;
    benchhw_*) v=${s#benchhw_}; export GPU_MAX_HW_QUEUES=${v%%_*}; step $s 300 python3 bench.py --no-corr --no-cpu-baseline --no-verify --steps 20; unset GPU_MAX_HW_QUEUES ;;
    benchq_*) export KRCA_PPR_GRID=${s#benchq_}; step $s 300 python3 bench.py --no-corr --no-cpu-baseline; unset KRCA_PPR_GRID ;;
    smoke) step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    bench_trace) prof bench_trace 400 bench.py --steps 10 --warmup 2 --no-cpu-baseline ;;
    bench_trace_full) prof bench_trace_full 700 bench.py ;;
    corr100k) prof corr100k 300 tools/prof_kernels.py corr --pods 100000 --reps 3 --tau 0.5 ;;
    corr100k_w*) export KRCA_LIB=$PWD/kubernetes-rca-system_amd/lib/libkrca_${s#corr100k_}.so; prof $s 300 tools/prof_kernels.py corr --pods 100000 --reps 3 --tau 0.5; unset KRCA_LIB ;;
    corrg_*) v=${s#corrg_}; export KRCA_CORR_RS_GROUP=${v%%_*}; prof $s 300 tools/prof_kernels.py corr --pods 100000 --reps 3 --tau 0.5; unset KRCA_CORR_RS_GROUP ;;
    corr1mg_*) v=${s#corr1mg_}; export KRCA_CORR_RS_GROUP=${v%%_*}; step $s 300 python3 tools/prof_kernels.py corr --pods 1000000 --reps 1 --tau 0.5; unset KRCA_CORR_RS_GROUP ;;
    corr1m) prof corr1m 600 tools/prof_kernels.py corr --pods 1000000 --reps 1 --tau 0.5 ;;
    corr_batch)  # C3 with the main pass in smaller batches: re-scores of batch b beside the tiles of b + 1
      for b in 128 256 512; do
        export KRCA_CORR_BATCH=$b; step corr_batch$b 300 python3 tools/prof_kernels.py corr --pods 100000 --reps 3 --tau 0.5
      done; unset KRCA_CORR_BATCH ;;
    ranking) step ranking 600 python3 -u tools/ranking_ablation_c4.py --seeds 2 --out $O/ranking_ablation_c4.json ;;
    ranking_spread) step ranking_spread 900 python3 -u tools/ranking_ablation_c4.py --seeds 2 --spread --out $O/ranking_ablation_spread_c4.json ;;
    ppr) prof ppr 300 tools/prof_kernels.py ppr --reps 5 ;;
    ppr_g8) step ppr_g8 300 python3 tools/ppr_g8_emulation.py ;;
    log_timing) export KRCA_LOG_FUSED=1 KRCA_LIB=$PWD/kubernetes-rca-system_amd/lib/libkrca_ltime.so; step log_timing 300 python3 tools/log_timing.py; unset KRCA_LIB KRCA_LOG_FUSED ;;
    diag_window) step diag_window 300 python3 -u tools/diag_window_templates.py ;;
    g8_step) step g8_step 400 python3 tools/g8_step_emulation.py ;;
    g8_dec) step g8_dec 500 python3 tools/g8_step_emulation.py --decoupled 1.0,1.5,2.0 ;;
    g8_dec_w*) step $s 500 python3 tools/g8_step_emulation.py --world ${s#g8_dec_w} --steps 30 --reps 5 --decoupled 1.0,1.5 ;;
    g8_slack_w*) step $s 500 python3 tools/g8_step_emulation.py --world ${s#g8_slack_w} --steps 30 --reps 5 --decoupled 1.25,1.5,2.0,3.0 ;;
    g8_rep_w*) step $s 500 python3 tools/g8_step_emulation.py --world ${s#g8_rep_w} --steps 30 --reps 5 --decoupled 1.5 --with-replicated ;;
    g8_roles_w*) step $s 500 python3 tools/g8_step_emulation.py --world ${s#g8_roles_w} --steps 30 --reps 5 --decoupled 1.5 --roles --hw-queues 16 ;;
    g8_grid_*) v=${s#g8_grid_}; step $s 500 python3 tools/g8_step_emulation.py --world 8 --steps 30 --reps 5 --decoupled 1.5 --hw-queues 16 --grid ${v%%_*} ;;
    g8_hq_w*) step $s 500 python3 tools/g8_step_emulation.py --world ${s#g8_hq_w} --steps 30 --reps 5 --decoupled 1.5 --with-replicated --hw-queues 16 ;;
    g8_grid) step g8_grid 400 python3 tools/g8_step_emulation.py --ppr-grids 0,1024,512,256 --only-grids ;;
    ppr_head)  # the same profile with the committed tree's code (ab_head/: git archive HEAD, built in place)
      step ppr_head 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ppr_head -o run -- python3 ab_head/tools/prof_kernels.py ppr --reps 5 ;;
    ppr_bytes) step ppr_bytes 300 python3 tools/ppr_bench.py --reps 5 ;;
    ppr_fuse) export KRCA_PPR_FUSE=1; prof ppr_fuse 300 tools/prof_kernels.py ppr --reps 5; unset KRCA_PPR_FUSE ;;
    ppr_timing) export KRCA_LIB=$PWD/kubernetes-rca-system_amd/lib/libkrca_ptime.so PPR_TIMING_DUMP=$O/ppr_timing.npz; step ppr_timing 300 python3 tools/ppr_timing.py; unset KRCA_LIB PPR_TIMING_DUMP ;;
    ppr_w*) export KRCA_LIB=$PWD/kubernetes-rca-system_amd/lib/libkrca_${s#ppr_}.so; prof $s 300 tools/prof_kernels.py ppr --reps 5; unset KRCA_LIB ;;
    ppr_prev) export KRCA_LIB=$PWD/kubernetes-rca-system_amd/lib/libkrca_prev.so; prof ppr_prev 300 tools/prof_kernels.py ppr --reps 5; unset KRCA_LIB ;;
    ppr_nt) export KRCA_PPR_NT=1; prof ppr_nt 300 tools/prof_kernels.py ppr --reps 5; unset KRCA_PPR_NT ;;
    bench_nograph) export KRCA_RCA_GRAPH=0; step bench_nograph 300 python3 bench.py --no-cpu-baseline; unset KRCA_RCA_GRAPH ;;
    bench2) step bench2 300 python3 bench.py --no-cpu-baseline ;;
    tests_tmpl) step tests_tmpl 600 python3 -u -m pytest tests -m gpu -x -v -rP --timeout 240 --timeout-method thread -k "template or tmpl or c2mini or c5 or stream" ;;
    logs) prof logs 300 tools/prof_kernels.py logs --reps 5 ;;
    logs_w*) export KRCA_LIB=$PWD/kubernetes-rca-system_amd/lib/libkrca_${s#logs_}.so; prof $s 300 tools/prof_kernels.py logs --reps 5; unset KRCA_LIB ;;
    tmpl) prof tmpl 300 tools/prof_kernels.py tmpl --reps 5 ;;
    tmpl_w*) export KRCA_LIB=$PWD/kubernetes-rca-system_amd/lib/libkrca_${s#tmpl_}.so; prof $s 300 tools/prof_kernels.py tmpl --reps 5; unset KRCA_LIB ;;
    c5) step c5 400 python3 -u tools/bench_stream.py ;;
    c5_phases) step c5_phases 400 python3 -u tools/bench_stream.py --phases ;;
    c5_trace) step c5_trace 400 rocprofv3 --kernel-trace --output-format csv -d $O/c5_trace -o run -- python3 -u tools/bench_stream.py --windows 4
      python3 tools/trace_gaps.py $O/c5_trace/run_kernel_trace.csv > $O/c5_gaps.txt; rm -f $O/c5_trace/run_kernel_trace.csv ;;
    pmc_ppr)
      pmc pmc_ppr_sq ppr SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
      pmc pmc_ppr_sq2 ppr SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD
      pmc pmc_ppr_tcc ppr TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum
      pmc pmc_ppr_tcp ppr TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
      pmc pmc_ppr_ea ppr TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum
      pmc pmc_ppr_grbm ppr GRBM_GUI_ACTIVE GRBM_COUNT ;;
    pmc_ppr_dram) pmc pmc_ppr_dram ppr TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum ;;
    pmc_logs_ea) pmc pmc_logs_ea logs TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum ;;
    pmc_logs_ea_w*) export KRCA_LIB=$PWD/kubernetes-rca-system_amd/lib/libkrca_${s#pmc_logs_ea_}.so
      pmc $s logs TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum; unset KRCA_LIB ;;
    pmc_logs)
      pmc pmc_logs_ea logs TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum
      pmc pmc_logs_sq logs SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo all-done >> $O/status
