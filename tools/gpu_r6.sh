#!/bin/bash
# Round-6 GPU call: named steps, each under its own time limit, stopping at the first failure.
# usage: tools/gpu_r6.sh TAG step [step ...]
#   tests        all -m gpu tests                    tests_K      -m gpu tests matching -k K
#   bench        bench.py default line               bench_trace  rocprofv3 stats of bench.py
#   smoke        __graft_entry__.smoke()             bench_cpufull  the CPU baseline also over every pod
#   rank_M       tools/ranking_ablation_c4.py --model M (C4, 2 seeds; M = default, spread, chain)
#   ppr          rocprofv3 stats of the C4 PageRank propagate   logs / tmpl  same for logs / templates
#   corr100k / corr1m   rocprofv3 stats of the correlation at C3 / 1M pods (tau 0.5)
#   c5           tools/bench_stream.py (C5 window)   g8           tools/g8_step_emulation.py --decoupled
#   graphprobe_J_N / graphprobeoff_J_N  tools/graph_replay_probe.py (--junk J --launches N) with packet capture on / off
#   tmplcls      template tests + kernel stats with the byte-class table build (lib/dbg/libkrca_tcls.so)
#   tmplr5       template kernel stats with the round-5 hash kernel (lib/dbg/libkrca_tr5.so; its hashes ignore UUIDs)
#   pmclds_V_T   LDS / issue counters of prof_kernels.py T (V = base or cls: the library)
#   pmcldsf_T    the same with KRCA_LOG_FUSED=2 (+ GRBM_GUI_ACTIVE)    logsf  logs stats with KRCA_LOG_FUSED=2
#   ltime_F      tools/log_timing.py (phase cycles per tile) with KRCA_LOG_FUSED=F and the -DLOG_TIMING build
#   pmcmfma      tools/gpu_pmc_mfma.sh (correlation MFMA busy, clock, DRAM bytes at C3 / 1M)
#   pmcx_T       tools/gpu_pmc_exact.sh with TARGETS=T (one target: cal ppr bench logs tmpl ...)
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
  # testsall_*: failing tests (pytest rc 1) do not stop the call; a timeout, crash or fault does
  if [ $rc -eq 1 ] && [ "${name#testsall_}" != "$name" ]; then tail -5 $O/$name.log; return 0; fi
  [ $rc -eq 0 ] || { echo "stop after $name"; tail -30 $O/$name.log; exit $rc; }
  tail -3 $O/$name.log
}
prof() {  # prof NAME SECONDS ARGS... (rocprofv3 kernel-trace stats of python3 ARGS)
  local name=$1 secs=$2; shift 2
  step $name $secs rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- python3 "$@"
}
for s in "$@"; do
  case $s in
    tests) step tests 900 python3 -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread ;;
    testsall_*) step $s 900 python3 -u -m pytest tests -m gpu -v -rP --timeout 300 --timeout-method thread -k "${s#testsall_}" ;;
    tests_*) step $s 900 python3 -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread -k "${s#tests_}" ;;
    bench) step bench 400 python3 bench.py ;;
    benchgraph_*) step $s 400 env KRCA_RCA_GRAPH=1 python3 bench.py --no-corr --no-cpu-baseline ;;
    bencheager_*) step $s 400 python3 bench.py --no-corr --no-cpu-baseline ;;
    bench8gloo) step bench8gloo 900 env KRCA_BENCH_BACKEND=gloo python3 bench.py --gpus 8 --steps 3 --warmup 1 --no-corr --no-cpu-baseline ;;
    bench8gloobal) step bench8gloobal 900 env KRCA_BENCH_BACKEND=gloo python3 bench.py --gpus 8 --steps 3 --warmup 1 --no-corr --no-cpu-baseline --ppr-partition balanced ;;
    smoke) step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    graphdbg) step testsall_graphdbg 300 python3 -u -m pytest tests -m gpu -v -rP --timeout 120 --timeout-method thread -k "replay_after or graph" ;;
    bench_cpufull) step bench_cpufull 500 python3 bench.py --steps 3 --warmup 1 --cpu-full-mesh --no-corr ;;
    bench_trace) prof bench_trace 500 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-verify ;;
    rank_*) m=${s#rank_}; step $s 900 python3 -u tools/ranking_ablation_c4.py --model $m --out $O/ranking_ablation_${m}_c4.json ;;
    ppr) prof ppr 300 tools/ppr_bench.py --reps 10 ;;
    logs) prof logs 300 tools/prof_kernels.py logs --reps 5 ;;
    tmpl) prof tmpl 300 tools/prof_kernels.py tmpl --reps 5 ;;
    corr100k) prof corr100k 400 tools/prof_kernels.py corr --pods 100000 --reps 3 ;;
    corr1m) prof corr1m 600 tools/prof_kernels.py corr --pods 1000000 --reps 1 ;;
    corrdbg_*) v=${s#corrdbg_}; export KRCA_CORR_DEBUG=${v%%_*}; prof $s 400 tools/prof_kernels.py corr --pods ${P:-1000000} --reps 1 --tau ${v##*_}; unset KRCA_CORR_DEBUG ;;
    corrside_*) v=${s#corrside_}; export KRCA_CORR_SIDE=${v%%_*}; prof $s 400 tools/prof_kernels.py corr --pods ${v##*_} --reps 3 --tau 0.5; unset KRCA_CORR_SIDE ;;
    corrkm_*) v=${s#corrkm_}; export KRCA_CORR_KM_EXTRA=${v%%_*}; prof $s 400 tools/prof_kernels.py corr --pods ${v##*_} --reps 3 --tau 0.5; unset KRCA_CORR_KM_EXTRA ;;
    corrbatch_*) v=${s#corrbatch_}; export KRCA_CORR_BATCH=${v%%_*}; prof $s 400 tools/prof_kernels.py corr --pods ${v##*_} --reps 3 --tau 0.5; unset KRCA_CORR_BATCH ;;
    corrrsg_*) v=${s#corrrsg_}; export KRCA_CORR_RSG_GRID=${v%%_*}; prof $s 400 tools/prof_kernels.py corr --pods ${v##*_} --reps 1 --tau 0.5; unset KRCA_CORR_RSG_GRID ;;
    pmcsq_*) t=${s#pmcsq_}; step $s 150 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O/$s -o run -- python3 tools/prof_kernels.py $t --reps 1 ;;
    c5) step c5 400 python3 tools/bench_stream.py ;;
    tmplcls) step tests_tmplcls 300 env KRCA_LIB=kubernetes-rca-system_amd/lib/dbg/libkrca_tcls.so python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "template or c5" &&
             KRCA_LIB=$PWD/kubernetes-rca-system_amd/lib/dbg/libkrca_tcls.so prof tmplcls 300 tools/prof_kernels.py tmpl --reps 5 ;;
    tmplr5) KRCA_LIB=$PWD/kubernetes-rca-system_amd/lib/dbg/libkrca_tr5.so prof tmplr5 300 tools/prof_kernels.py tmpl --reps 5 ;;
    pmclds_*) t=${s#pmclds_}; lib=""; [ "${t%%_*}" = cls ] && lib=$PWD/kubernetes-rca-system_amd/lib/dbg/libkrca_tcls.so; t=${t#*_};
              step $s 150 env ${lib:+KRCA_LIB=$lib} timeout -s KILL 140 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O/$s -o run -- python3 tools/prof_kernels.py $t --reps 1 ;;
    pmcldsf_*) t=${s#pmcldsf_}; step $s 150 env KRCA_LOG_FUSED=2 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/$s -o run -- python3 tools/prof_kernels.py $t --reps 1 ;;
    logsf) step logsf 300 env KRCA_LOG_FUSED=2 rocprofv3 --kernel-trace --stats --output-format csv -d $O/logsf -o run -- python3 tools/prof_kernels.py logs --reps 5 ;;
    ltime_*) step $s 300 env KRCA_LOG_FUSED=${s#ltime_} KRCA_LIB=$PWD/kubernetes-rca-system_amd/lib/dbg/libkrca_ltime.so python3 -u tools/log_timing.py ;;
    graphprobe_*) v=${s#graphprobe_}; step $s 300 env KRCA_LIB=kubernetes-rca-system_amd/lib/dbg/libkrca_gdbg.so python3 -u tools/graph_replay_probe.py --junk ${v%%_*} --launches ${v##*_} ;;
    graphprobeoff_*) v=${s#graphprobeoff_}; step $s 300 env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 KRCA_LIB=kubernetes-rca-system_amd/lib/dbg/libkrca_gdbg.so python3 -u tools/graph_replay_probe.py --junk ${v%%_*} --launches ${v##*_} ;;
    pmcmfma) step pmcmfma 1000 env PODS="${PODS:-100000 1000000}" tools/gpu_pmc_mfma.sh $TAG/pmcmfma ;;
    pmcx_*) step $s 1000 env TARGETS="${s#pmcx_}" tools/gpu_pmc_exact.sh $TAG/$s ;;
    cumask) step cumask 600 python3 -u tools/cu_mask_probe.py ;;
    prio) step prio 600 python3 -u tools/cu_mask_probe.py --prio-only --steps 20 ;;
    scoreab_*) step $s 400 python3 -u tools/score_ab.py --pods ${s#scoreab_} --only pipe_c10,pipe_c12,pipe_c15,pipe_c20,pipe_c30,ring_buf --rounds 3 --reps 5 ;;
    g8slack_*) step $s 700 python3 -u tools/g8_step_emulation.py --world ${s#g8slack_} --decoupled 1.25,1.5,2.0 --reps 5 --hw-queues 16 --steps 30 ;;
    g8grid_*) step $s 700 python3 -u tools/g8_step_emulation.py --world 8 --decoupled 1.5 --reps 5 --hw-queues 16 --steps 30 --grid ${s#g8grid_} ;;
    g8_*) step $s 700 python3 -u tools/g8_step_emulation.py --world ${s#g8_} --decoupled 1.5 --reps 5 --with-replicated --hw-queues 16 --steps 30 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
