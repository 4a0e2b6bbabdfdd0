#!/bin/bash
# One GPU call made of named steps, run in order; the first failing step ends the call (no GPU step
# after a failure, a fault or a time limit).  Replaces round 4's one-off tools/gpu_r04*.sh scripts.
# Usage (repo root, on the GPU box):  bash tools/gpu_job.sh <tag> <step> [<step> ...]
#   smoke             __graft_entry__.smoke()
#   tests[:<k-expr>]  pytest -m gpu (error census in flips.jsonl / tol.jsonl; -k <k-expr> if given)
#   bench             the default bench line (with its CPU baseline) + tools/bench_summary.py
#   benchq            the default bench line without the CPU baseline
#   ab:<lib>          bench line of an alternative libflsim.so (FLSIM_LIB=<lib>) beside benchq
#   abvgg:<lib>       configs[4] (vgg11, n = 4096, d = 1000) with an alternative libflsim.so, B A B A
#   bl:<name>:<lib>  one bench line on another libflsim.so build (FLSIM_LIB)
#   ltests:<lib>:<k> pytest -m gpu -k <k> on another build (tol_<build>.jsonl)
#   abenv:<VAR=VAL>   bench line with one environment setting beside benchq (E1 A1 E2 A2)
#   c1abenv:<VAR=VAL> the same on configs[1] (n = 10, d = 50, the warm start)
#   trace             rocprofv3 --kernel-trace --stats of a short bench (kernel_stats.csv)
#   pmc               FETCH/WRITE + two SQ passes on one 128-worker chunk, traffic table, summary
#   tatd              TA / TD / TCP passes on one 128-worker chunk (tools/pmc_summary_ta.py)
#   lds               LDS / VMEM issue passes on one 128-worker chunk (tools/pmc_summary.py)
#   gloo2             2-rank gloo rehearsal of the N > 1 path through bench.py (n = 256)
#   forcedist         torchrun --nproc-per-node 1 bench.py --force-dist (RCCL at world size 1)
#   sizes             the per-rank loads of an N-GPU job on one GPU: n = 128 / 256 / 512
#   fwd1              tools/fwd1_bench.py (the facade's one-call forward alone)
#   aggceil           tools/agg_ceiling.py (torch streams at the aggregation paths' sizes)
#   facadeab:<VAR=VAL> the facade loop with one environment setting, E A E A
#   facade            tools/facade_bench.py (the FL.agents reference loop, n = 1024)
#   vfacadeab:<VAR=VAL> the same loop with vgg11, one environment setting, E A E A (bfacadeab: vgg11_bn)
#   configs           tools/gpu_configs_all.sh (the other BASELINE configs)
#   lab:<bin>[:<arg>] a lab binary from tools/lab (built beforehand on the CPU)
#   labab:<b0>:<b1>:<arg>  two lab binaries A B A B on the same box
#   diag[:<pkg>]      tools/survey_diag.py (SURVEY 8(c) per tensor; <pkg>: another build's flsim)
#   gemmdiag          tools/gemm_diag.py for the conv6 / conv5 / conv4 data-gradient GEMMs
#   facadetrace       rocprofv3 kernel trace of tools/facade_bench.py + tools/trace_gaps.py
#   streampmc         SQ counters of the post-all-reduce stream (tools/agg_bench.py, tools/stream_pmc.py)
#   c1trace           rocprofv3 kernel trace of configs[1] (n = 10, warm start) + tools/trace_gaps.py
set -u
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
KREGEX="gemm_kernel|gemm_x6_kernel|gemm_dx6_kernel|gemm_direct_kernel|gemm_halo|k_conv1_fwd|k_slab_step|k_pool_scatter|k_agg_stream"
CHUNK="--n_workers 128 --no-throttle --steps 1 --warmup 0 --no-cpu-baseline --no-probe --no-stream"

pmc_passes() {   # <dir> <pass>... : one counter group per rocprofv3 run over one 128-worker chunk
    local d=$1; shift
    local i=0
    for PASS in "$@"; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --pmc $PASS --output-format csv -d $d/p$i -o run \
            --kernel-include-regex "$KREGEX" -- python3 bench.py $CHUNK > $d/p$i.log 2>&1 \
            || { echo "pass $i ($PASS) failed $?"; tail -5 $d/p$i.log; exit 1; }
        echo "pass $i ok: $PASS"
    done
}

bench_line() {   # <name> [env...] : one bench line without the CPU baseline ($BENCH_ARGS appended)
    local name=$1; shift
    env "$@" timeout -k 10 400 python3 -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench_$name.json \
        2> $OUT/bench_$name.err || { echo "bench $name failed $?"; tail -5 $OUT/bench_$name.err; exit 1; }
    python3 tools/bench_summary.py $OUT/bench_$name.json > $OUT/bench_$name.txt
    echo "$name: $(head -1 $OUT/bench_$name.txt)"
}

for STEP in "$@"; do
    case $STEP in
    smoke)
        timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 \
            || { echo "smoke failed $?"; tail -5 $OUT/smoke.txt; exit 1; }
        tail -1 $OUT/smoke.txt ;;
    tests|tests:*)
        K=${STEP#tests}; K=${K#:}
        FLSIM_FLIP_LOG=$OUT/flips.jsonl FLSIM_TOL_LOG=$OUT/tol.jsonl timeout -k 10 1000 python3 -u \
            -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread ${K:+-k "$K"} \
            > $OUT/pytest_gpu.txt 2>&1
        rc=$?
        tail -2 $OUT/pytest_gpu.txt; grep -E "^FAILED" $OUT/pytest_gpu.txt | head
        [ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; exit $rc; } ;;
    bench)
        timeout -k 10 400 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err \
            || { echo "bench failed $?"; tail -5 $OUT/bench.err; exit 1; }
        python3 tools/bench_summary.py $OUT/bench.json > $OUT/bench.txt
        head -3 $OUT/bench.txt ;;
    benchq)
        bench_line q ;;
    ab:*)
        LIB=${STEP#ab:}
        bench_line B1 FLSIM_LIB=$LIB; bench_line A1; bench_line B2 FLSIM_LIB=$LIB; bench_line A2 ;;
    c1abenv:*)
        KV=${STEP#c1abenv:}
        timeout -k 10 120 python -u tools/warm_start_file.py --out $OUT/warm_start.pt > $OUT/c1_warm.log 2>&1 \
            || { echo "warm start failed"; exit 1; }
        BENCH_ARGS="--n_workers 10 --delay 50 --model_file $OUT/warm_start.pt --steps 200 --warmup 10"
        bench_line c1E1 $KV; bench_line c1A1; bench_line c1E2 $KV; bench_line c1A2
        BENCH_ARGS="" ;;
    abvgg:*)
        LIB=${STEP#abvgg:}
        BENCH_ARGS="--model vgg11 --n_workers 4096 --delay 1000 --steps 4 --warmup 1"
        bench_line vB1 FLSIM_LIB=$LIB; bench_line vA1; bench_line vB2 FLSIM_LIB=$LIB; bench_line vA2
        BENCH_ARGS="" ;;
    bl:*)          # bl:<name>:<lib> one bench line on another build of libflsim.so
        SPEC=${STEP#bl:}; bench_line ${SPEC%%:*} FLSIM_LIB=${SPEC#*:} ;;
    ltests:*)      # ltests:<lib>:<k-expr> pytest -m gpu -k <k-expr> on another build
        SPEC=${STEP#ltests:}; LIB=${SPEC%%:*}; K=${SPEC#*:}; N=$(basename $(dirname $LIB))
        FLSIM_LIB=$LIB FLSIM_TOL_LOG=$OUT/tol_$N.jsonl timeout -k 10 1000 python3 -u \
            -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread -k "$K" \
            > $OUT/pytest_$N.txt 2>&1
        rc=$?
        tail -2 $OUT/pytest_$N.txt; grep -E "^FAILED" $OUT/pytest_$N.txt | head
        [ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; exit $rc; } ;;
    abenv:*)
        KV=${STEP#abenv:}
        bench_line E1 $KV; bench_line A1; bench_line E2 $KV; bench_line A2 ;;
    trace)
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
            -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stream > $OUT/trace.log 2>&1 \
            || { echo "trace failed $?"; tail -5 $OUT/trace.log; exit 1; }
        cp $(find $OUT/trace -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
        echo "trace ok" ;;
    pmc)
        D=$OUT/pmc; mkdir -p $D
        pmc_passes $D "FETCH_SIZE" "WRITE_SIZE" \
          "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS" \
          "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
        TR=$D/traffic_in
        mkdir -p $TR/pmc_FETCH_SIZE $TR/pmc_WRITE_SIZE $TR/trace
        cp $(find $D/p1 -name "*counter_collection.csv" | head -1) $TR/pmc_FETCH_SIZE/run_counter_collection.csv
        cp $(find $D/p2 -name "*counter_collection.csv" | head -1) $TR/pmc_WRITE_SIZE/run_counter_collection.csv
        if [ -f $OUT/kernel_stats.csv ]; then cp $OUT/kernel_stats.csv $TR/trace/run_kernel_stats.csv; fi
        python3 tools/pmc_traffic.py $TR $D/traffic.json > $D/traffic.txt && cat $D/traffic.txt
        python3 tools/pmc_summary.py $D > $D/summary.txt && cat $D/summary.txt ;;
    tatd)
        D=$OUT/tatd; mkdir -p $D
        pmc_passes $D "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
          "TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
          "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
        python3 tools/pmc_summary_ta.py $D > $D/summary.txt && cat $D/summary.txt ;;
    lds)
        D=$OUT/lds; mkdir -p $D
        pmc_passes $D \
          "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
          "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY"
        python3 tools/pmc_summary.py $D > $D/summary.txt && cat $D/summary.txt ;;
    gloo2)
        timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
            --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --backend gloo \
            --n_workers 256 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_n2_gloo.json \
            2> $OUT/bench_n2_gloo.err || { echo "gloo rehearsal failed $?"; tail -5 $OUT/bench_n2_gloo.err; exit 1; }
        cut -c1-200 $OUT/bench_n2_gloo.json ;;
    forcedist)
        timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
            --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 1 --force-dist \
            --backend nccl --no-cpu-baseline > $OUT/bench_forcedist.json 2> $OUT/bench_forcedist.err \
            || { echo "forcedist failed $?"; tail -8 $OUT/bench_forcedist.err; exit 1; }
        python3 tools/bench_summary.py $OUT/bench_forcedist.json > $OUT/bench_forcedist.txt
        head -3 $OUT/bench_forcedist.txt ;;
    sizes)
        for N in 128 256 512; do
            timeout -k 10 300 python3 -u bench.py --n_workers $N --no-cpu-baseline --no-stream \
                > $OUT/bench_n$N.json 2> $OUT/bench_n$N.err || { echo "n=$N failed $?"; exit 1; }
            python3 tools/bench_summary.py $OUT/bench_n$N.json > $OUT/bench_n$N.txt
            echo "n=$N: $(head -1 $OUT/bench_n$N.txt)"
        done ;;
    fwd1)
        timeout -k 10 200 python3 -u tools/fwd1_bench.py > $OUT/fwd1.json 2> $OUT/fwd1.err \
            || { echo "fwd1 failed $?"; tail -5 $OUT/fwd1.err; exit 1; }
        cat $OUT/fwd1.json ;;
    fwd1trace)
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/f1trace -o run \
            -- python3 tools/fwd1_bench.py --calls 200 > $OUT/fwd1_trace.log 2>&1 \
            || { echo "fwd1 trace failed $?"; tail -5 $OUT/fwd1_trace.log; exit 1; }
        D=$(dirname $(find $OUT/f1trace -name "run_kernel_trace.csv" | head -1))
        cp $D/run_kernel_stats.csv $OUT/fwd1_kernel_stats.csv
        python3 tools/trace_gaps.py $D 0.5 > $OUT/fwd1_gaps.txt && head -40 $OUT/fwd1_gaps.txt ;;
    aggceil)
        timeout -k 10 300 python3 -u tools/agg_ceiling.py > $OUT/agg_ceiling.txt 2>&1 \
            || { echo "agg ceiling failed $?"; tail -5 $OUT/agg_ceiling.txt; exit 1; }
        cat $OUT/agg_ceiling.txt ;;
    facade)
        timeout -k 10 600 python3 -u tools/facade_bench.py --epochs 6 > $OUT/facade_bench.json 2> $OUT/facade_bench.err \
            || { echo "facade failed $?"; tail -5 $OUT/facade_bench.err; exit 1; }
        cut -c1-400 $OUT/facade_bench.json ;;
    streampmc)
        D=$OUT/streampmc; mkdir -p $D
        timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE \
            --output-format csv -d $D/p1 -o run --kernel-include-regex "k_agg_stream|k_slab_step" \
            -- python3 tools/agg_bench.py --iters 5 > $D/p1.log 2>&1 || { echo "stream pmc failed $?"; tail -5 $D/p1.log; exit 1; }
        cp $(find $D/p1 -name "*counter_collection.csv" | head -1) $D/counters.csv
        python3 tools/stream_pmc.py $D/counters.csv | tee $D/summary.txt ;;
    c1trace)
        timeout -k 10 120 python -u tools/warm_start_file.py --out $OUT/warm_start.pt > $OUT/c1_warm.log 2>&1 \
            || { echo "warm start failed"; exit 1; }
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c1trace -o run \
            -- python3 bench.py --n_workers 10 --delay 50 --model_file $OUT/warm_start.pt --steps 40 \
            --warmup 5 --no-cpu-baseline > $OUT/c1trace.log 2>&1 \
            || { echo "configs1 trace failed $?"; tail -5 $OUT/c1trace.log; exit 1; }
        D=$(dirname $(find $OUT/c1trace -name "run_kernel_trace.csv" | head -1))
        cp $D/run_kernel_stats.csv $OUT/c1_kernel_stats.csv
        python3 tools/trace_gaps.py $D 0.5 > $OUT/c1_gaps.txt && head -30 $OUT/c1_gaps.txt ;;
    vfacadeab:*|bfacadeab:*)   # the vgg11 / vgg11_bn facade loop (n = 1024), one setting, E A E A
        KV=${STEP#?facadeab:}
        FM=vgg11; [ ${STEP:0:1} = b ] && FM=vgg11_bn
        for R in E1 A1 E2 A2; do
            if [ ${R:0:1} = E ]; then ENVS="$KV"; else ENVS="FLSIM_NOOP=1"; fi
            env $ENVS timeout -k 10 300 python3 -u tools/facade_bench.py --model $FM --epochs 4 \
                > $OUT/${FM}_facade_$R.json 2> $OUT/${FM}_facade_$R.err \
                || { echo "$FM facade $R failed $?"; tail -5 $OUT/${FM}_facade_$R.err; exit 1; }
            echo "$R $(cut -c1-130 $OUT/${FM}_facade_$R.json)"
        done ;;
    facadeab:*)
        KV=${STEP#facadeab:}
        for R in E1 A1 E2 A2; do
            if [ ${R:0:1} = E ]; then ENVS="$KV"; else ENVS="FLSIM_NOOP=1"; fi
            env $ENVS timeout -k 10 300 python3 -u tools/facade_bench.py --epochs 4 > $OUT/facade_$R.json \
                2> $OUT/facade_$R.err || { echo "facade $R failed $?"; tail -5 $OUT/facade_$R.err; exit 1; }
            echo "$R $(cut -c1-120 $OUT/facade_$R.json)"
        done ;;
    facadetrace)
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ftrace -o run \
            -- python3 tools/facade_bench.py --epochs 2 > $OUT/facade_trace.log 2>&1 \
            || { echo "facade trace failed $?"; tail -5 $OUT/facade_trace.log; exit 1; }
        D=$(dirname $(find $OUT/ftrace -name "run_kernel_trace.csv" | head -1))
        cp $D/run_kernel_stats.csv $OUT/facade_kernel_stats.csv
        python3 tools/trace_gaps.py $D 0.5 > $OUT/facade_gaps.txt && head -30 $OUT/facade_gaps.txt ;;
    configs)
        bash tools/gpu_configs_all.sh $TAG || exit 1 ;;
    labenv:*)      # labenv:<VAR=VAL>:<bin>[:<arg>]
        SPEC=${STEP#labenv:}; KV=${SPEC%%:*}; SPEC=${SPEC#*:}; BIN=${SPEC%%:*}; ARG=${SPEC#$BIN}; ARG=${ARG#:}
        env $KV timeout -k 10 300 tools/lab/$BIN $ARG > $OUT/lab_$BIN.txt 2>&1 \
            || { echo "lab $BIN failed $?"; tail -5 $OUT/lab_$BIN.txt; exit 1; }
        cat $OUT/lab_$BIN.txt ;;
    lab:*)
        SPEC=${STEP#lab:}; BIN=${SPEC%%:*}; ARG=${SPEC#$BIN}; ARG=${ARG#:}
        timeout -k 10 300 tools/lab/$BIN $ARG > $OUT/lab_$BIN${ARG:+_$ARG}.txt 2>&1 \
            || { echo "lab $BIN failed $?"; tail -5 $OUT/lab_$BIN*.txt; exit 1; }
        cat $OUT/lab_$BIN${ARG:+_$ARG}.txt ;;
    labab:*)
        IFS=: read -r _ B0 B1 ARG <<< "$STEP"
        for r in 1 2; do
            for B in $B0 $B1; do
                timeout -k 10 300 tools/lab/$B $ARG > $OUT/labab_${B}_$r.txt 2>&1 \
                    || { echo "lab $B failed $?"; tail -5 $OUT/labab_${B}_$r.txt; exit 1; }
                sed "s/^/$B $r | /" $OUT/labab_${B}_$r.txt
            done
        done ;;
    diag|diag:*)
        PKG=${STEP#diag}; PKG=${PKG#:}
        NAME=diag_$(basename ${PKG:-tree})
        for IT in "0,1,2" "1,0,3 1,2,0"; do
            timeout -k 10 300 python3 -u tools/survey_diag.py ${PKG:+--pkg $PKG} --items $IT \
                >> $OUT/$NAME.txt 2>&1 || { echo "diag failed $?"; tail -5 $OUT/$NAME.txt; exit 1; }
        done
        grep -v SURVEY_DIAG $OUT/$NAME.txt ;;
    gemmdiag)
        for ST in 6 5 4; do
            FLSIM_DEBUG_BWD_STOP=$ST timeout -k 10 300 python3 -u tools/gemm_diag.py >> $OUT/gemm_diag.txt 2>&1 \
                || { echo "gemm diag $ST failed $?"; tail -5 $OUT/gemm_diag.txt; exit 1; }
        done
        grep GEMM_DIAG $OUT/gemm_diag.txt ;;
    *)
        echo "unknown step $STEP"; exit 2 ;;
    esac
done
echo "$TAG-ok"
