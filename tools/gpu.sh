#!/bin/bash
# One parameterised recipe for the GPU box (replaces the per-session tools/gpu_r0*.sh scripts).
#
#   tools/gpu.sh <tag> <step> [<step> ...]        (from the repo root)
#
# Output goes to gpurun_out/<tag>/.  Steps run in order, each under its own time limit; the first
# failing step ends the run (nothing further touches the GPU after a failure).
#
#   tests[=<pytest -k expr>]   the -m gpu suite (or the matching subset), one process
#   smoke                      __graft_entry__.smoke()
#   bench[=<extra args>]       bench.py --steps 20 --warmup 5 (the driver command) -> bench.json
#   trace[=<extra args>]       rocprofv3 --kernel-trace --stats over that bench command
#                              -> kernels.csv (per kernel+grid: launches, avg, median) + kernel_stats.csv
#   headline                   the same trace over the headline leg alone (no JPEG / configs /
#                              latency / CPU legs): the K2 average is the timed kernel's
#   ptrace=<probe>             kernel trace of one probe (c3 c5 jpeg png) -> <probe>_kernels.csv
#   pmc=<probe>                FETCH_SIZE / WRITE_SIZE passes over a probe -> pmc_traffic_<probe>.json
#   sq=<probe>                 SQ instruction / wait / LDS-conflict passes -> sq_<probe>.txt
#   py=<script> [args]         python3 tools/<script> [args] -> <script>.out
#   ab=<probe>:<v1>[,<v2>...]  same-box A/B/n: kernel traces of the probe with the in-tree libomr.so
#                              ("new") and ab/libomr_<v>.so (OMR_LIB; built by tools/ab_build.sh),
#                              alternated twice -> per-kernel medians in ab_<probe>.txt
set -o pipefail
TAG=${1:?tag}; shift
O=gpurun_out/$TAG; mkdir -p $O
R=$PWD
export TMPDIR=/tmp
export C5_TILES=${C5_TILES:-64} JPEG_PROBE_TILES=${JPEG_PROBE_TILES:-256}   # the bench's launch sizes

run() {   # run <seconds> <log> <cmd...>: one GPU step under its own limit; stop the script on failure
    local t=$1 log=$2; shift 2
    timeout -k 10 $t "$@" > $O/$log 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then echo "STEP FAILED rc=$rc: $*"; tail -30 $O/$log; exit $rc; fi
}

probe_cmd() {
    case $1 in
    c3) echo "python3 $R/tools/c3_probe.py" ;;
    c5) echo "python3 $R/tools/c5_probe.py" ;;
    jpeg) echo "python3 $R/tools/jpeg_probe.py" ;;
    png) echo "python3 $R/tools/png_batch_probe.py" ;;
    c2) echo "python3 $R/bench.py --steps 20 --warmup 5 --no-jpeg --no-configs --no-latency --no-cpu-baseline --prewarm-ms 50" ;;
    *) echo "unknown probe $1" >&2; exit 2 ;;
    esac
}

probe_regex() {
    case $1 in
    c3) echo "k_project" ;;
    c5|c2) echo "k_render" ;;
    jpeg) echo "k_jpeg|k_render" ;;
    png) echo "k_png" ;;
    esac
}

for step in "$@"; do
    name=${step%%=*}; arg=${step#*=}; [ "$arg" = "$step" ] && arg=""
    echo "== $step ($(date +%T))"
    case $name in
    tests)
        if [ -n "$arg" ]; then
            run 900 tests.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$arg"
        else
            run 1100 tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
        fi
        tail -3 $O/tests.log ;;
    smoke)
        run 300 smoke.log python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
        tail -1 $O/smoke.log ;;
    bench)
        timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 $arg > $O/bench.json 2> $O/bench.err \
            || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
        tail -c 400 $O/bench.json; echo ;;
    trace|headline)
        extra=$arg
        [ $name = headline ] && extra="--no-jpeg --no-configs --no-latency --no-cpu-baseline $arg"
        ( cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/t_$name -o t \
            -- python3 $R/bench.py --steps 20 --warmup 5 $extra ) > $O/${name}_bench.json 2> $O/$name.err \
            || { echo "$name trace failed"; tail -30 $O/$name.err; exit 1; }
        find $O/t_$name -name '*kernel_stats.csv' -exec cp {} $O/${name}_kernel_stats.csv \;
        f=$(find $O/t_$name -name '*kernel_trace.csv' | head -1)
        python3 tools/trace_kernels.py $f $O/${name}_kernels.csv && rm -rf $O/t_$name
        head -12 $O/${name}_kernels.csv | cut -c1-160 ;;
    ptrace)
        cmd=$(probe_cmd $arg) || exit 2
        ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pt_$arg -o t \
            -- $cmd ) > $O/ptrace_$arg.out 2> $O/ptrace_$arg.err \
            || { echo "ptrace $arg failed"; tail -30 $O/ptrace_$arg.err; exit 1; }
        f=$(find $O/pt_$arg -name '*kernel_trace.csv' | head -1)
        python3 tools/trace_kernels.py $f $O/${arg}_kernels.csv && rm -rf $O/pt_$arg
        head -20 $O/${arg}_kernels.csv | cut -c1-160 ;;
    pmc)
        cmd=$(probe_cmd $arg) || exit 2
        for c in FETCH_SIZE WRITE_SIZE; do
            ( cd /tmp && JPEG_PROBE_ITERS=2 timeout -s KILL 180 rocprofv3 --pmc $c --kernel-include-regex "$(probe_regex $arg)" \
                --output-format csv -d $R/$O/pmc_${arg}_$c -o p -- $cmd ) > /dev/null 2> $O/pmc_${arg}_$c.err \
                || { echo "pmc $arg $c failed"; tail -10 $O/pmc_${arg}_$c.err; exit 1; }
        done
        python3 tools/pmc_traffic.py $O/pmc_traffic_$arg.json $(find $O -path "*pmc_${arg}_*" -name '*counter_collection.csv') \
            > $O/pmc_traffic_$arg.txt || exit 1
        find $O -path "*pmc_${arg}_*" -name '*counter_collection.csv' -delete
        cat $O/pmc_traffic_$arg.txt | cut -c1-160 | head -30 ;;
    sq)
        cmd=$(probe_cmd $arg) || exit 2
        i=0
        for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_VALU_CVT" \
                   "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
                   "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
            i=$((i + 1))
            ( cd /tmp && JPEG_PROBE_ITERS=2 timeout -s KILL 180 rocprofv3 --pmc $grp --kernel-include-regex "$(probe_regex $arg)" \
                --output-format csv -d $R/$O/sq_${arg}/p$i -o p -- $cmd ) > /dev/null 2> $O/sq_${arg}_$i.err \
                || { echo "sq $arg pass $i failed"; tail -10 $O/sq_${arg}_$i.err; exit 1; }
        done
        python3 tools/pmc_kernels.py $(find $O/sq_$arg -name '*counter_collection.csv') > $O/sq_$arg.txt || exit 1
        python3 tools/sq_json.py $O/sq_$arg.txt $O/sq_$arg.json $TAG > /dev/null || exit 1
        if [ $arg = jpeg ]; then      # per-MCU form for bench.py's JPEG VALU roofline (1024^2 tiles: 4096 MCUs)
            python3 tools/pmc_kernels.py --json $O/jpeg_valu_pmc.json --case ${JPEG_PROBE_CASE:-c2} \
                --mcus $((JPEG_PROBE_TILES * 4096)) $(find $O/sq_$arg -name '*counter_collection.csv') > /dev/null || exit 1
        fi
        find $O/sq_$arg -name '*counter_collection.csv' -delete
        grep -E "==|VALU/wave|WAIT|BANK|IDX" $O/sq_$arg.txt | head -40 ;;
    ab)
        probe=${arg%%:*}; vars=${arg#*:}
        cmd=$(probe_cmd $probe) || exit 2
        for i in 1 2; do
            for v in new ${vars//,/ }; do
                if [ $v = new ]; then unset OMR_LIB; else export OMR_LIB=$R/ab/libomr_$v.so; fi
                ( cd /tmp && JPEG_PROBE_ITERS=${JPEG_PROBE_ITERS:-10} timeout -k 10 240 rocprofv3 --kernel-trace \
                    --output-format csv -d $R/$O/ab_$v$i -o t -- $cmd ) > $O/ab_$v$i.log 2>&1 \
                    || { echo "ab $v $i failed"; tail -20 $O/ab_$v$i.log; exit 1; }
                f=$(find $O/ab_$v$i -name '*kernel_trace.csv' | head -1)
                { echo "== $v $i"; python3 tools/trace_summary.py $f; } >> $O/ab_$probe.txt
                rm -rf $O/ab_$v$i
            done
        done
        unset OMR_LIB
        cat $O/ab_$probe.txt | cut -c1-120 ;;
    py)
        script=${arg%% *}; rest=${arg#"$script"}
        run 600 $(basename $script .py).out python3 -u tools/$script $rest
        tail -20 $O/$(basename $script .py).out ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
echo "GPU.SH $TAG OK"
