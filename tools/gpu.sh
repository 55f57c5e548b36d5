#!/bin/bash
# One parametrized GPU-box runner (replaces the round-3 single-experiment
# scripts).  Usage, through gpurun:
#   bash tools/gpu.sh TAG STEP [STEP ...]
# Steps run in order, each under its own timeout; the first failure ends the
# run (no GPU step after a failed one).  Output goes to gpurun_out/TAG/.
#   gputests            full `pytest -m gpu`
#   tests=EXPR          `pytest -m gpu -k EXPR`
#   smoke               __graft_entry__.smoke()
#   bench=ARGS          python bench.py ARGS        (ARGS: comma-separated, e.g. --general,only,--steps,10)
#   skew=ARGS           python tools/bench_skew.py ARGS
#   eskew=ENV/ARGS      tools/bench_skew.py ARGS with ENV (comma-separated K=V)
#   sskew=ARGS          tools/bench_skew.py ARGS with HPCJOIN_SHARE_GPU=1 (--gpus N: N RCCL ranks on this GPU)
#   phases=ARGS        tools/scatter_phases.py of the phase-stamped build in ab/prof (tools/README.md)
#   py=SCRIPT,ARGS      python SCRIPT ARGS
#   epy=ENV/SCRIPT,ARGS python SCRIPT ARGS with ENV (comma-separated K=V)
#   stats=ARGS          rocprofv3 --kernel-trace --stats of bench.py ARGS
#   estats=ENV/ARGS     the same with ENV exported (comma-separated K=V)
#   pstats=SCRIPT,ARGS  rocprofv3 --kernel-trace --stats of python SCRIPT ARGS
#   ppmc=CTRS/SCRIPT,ARGS  rocprofv3 --pmc CTRS of python SCRIPT ARGS
#   pmc=CTRS/ARGS       rocprofv3 --pmc CTRS (comma-separated) of bench.py ARGS
#   ebench=ENV/ARGS     bench.py ARGS with ENV (comma-separated K=V, e.g. HPCJOIN_NET_THREADS=512): A/B runs
#   abbench=ARGS        same-box A/B: bench.py ARGS of ab/base (a built copy of an older tree) and of this
#                       tree, alternating base/new twice
#   sweep=FIELD/V1:V2/ARGS  bench.py ARGS once per value of the HPCJOIN_<FIELD> override (parameter sweeps)
#   pmcset=GROUP/ARGS   a named PMC group of bench.py ARGS: fetch (FETCH_SIZE), write (WRITE_SIZE),
#                       sq (waves, busy/wait cycles, LDS instructions and bank conflicts, VMEM rd/wr)
#   rccl=N/ARGS         bench.py ARGS as N RCCL processes sharing this GPU (HPCJOIN_SHARE_GPU=1: socket
#                       transport -- the multi-process path end to end, not xGMI speed)
#   prccl=N/ARGS        the same under rocprofv3 --kernel-trace (stream overlap across ranks)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
TAG=$1
shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%=*}
  arg=${step#*=}
  [ "$arg" = "$step" ] && arg=""
  args=${arg//,/ }
  log=$OUT/$n.$kind.log
  echo "[$n] $step"
  case $kind in
    gputests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$log" 2>&1 ;;
    tests) timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$arg" > "$log" 2>&1 ;;
    smoke) timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > "$log" 2>&1 ;;
    bench) timeout -k 10 600 python -u bench.py $args > "$log" 2>&1 ;;
    ebench) envs=${arg%%/*}; bargs=${arg#*/}
            timeout -k 10 600 env ${envs//,/ } python -u bench.py ${bargs//,/ } > "$log" 2>&1 ;;
    skew) timeout -k 10 900 python -u tools/bench_skew.py $args > "$log" 2>&1 ;;
    eskew) envs=${arg%%/*}; sargs=${arg#*/}
           timeout -k 10 900 env ${envs//,/ } python -u tools/bench_skew.py ${sargs//,/ } > "$log" 2>&1 ;;
    phases) timeout -k 10 600 python -u ab/prof/tools/scatter_phases.py $args > "$log" 2>&1 ;;
    sskew) HPCJOIN_SHARE_GPU=1 timeout -k 10 900 python -u tools/bench_skew.py $args > "$log" 2>&1 ;;
    sweep) f=${arg%%/*}; rest=${arg#*/}; vals=${rest%%/*}; bargs=${rest#*/}; [ "$bargs" = "$rest" ] && bargs=""
           rc=0
           for v in ${vals//:/ }; do
             env HPCJOIN_$f=$v timeout -k 10 300 python -u bench.py ${bargs//,/ } > "$OUT/$n.$f=$v.log" 2>&1 || { rc=$?; break; }
           done
           echo "sweep $f rc=$rc" > "$log"; (exit $rc) ;;
    pmcset) grp=${arg%%/*}; bargs=${arg#*/}; [ "$bargs" = "$arg" ] && bargs=""
            case $grp in
              fetch) ctrs="FETCH_SIZE" ;;
              write) ctrs="WRITE_SIZE" ;;
              sq) ctrs="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" ;;
              *) echo "unknown pmc group $grp"; exit 2 ;;
            esac
            (cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $ctrs -d "$OUT/pmc$n" -o run \
               --output-format csv -- python "$R/bench.py" ${bargs//,/ }) > "$log" 2>&1 ;;
    rccl) np=${arg%%/*}; bargs=${arg#*/}; [ "$bargs" = "$arg" ] && bargs=""
          HPCJOIN_SHARE_GPU=1 timeout -k 10 900 python -u bench.py --gpus $np ${bargs//,/ } > "$log" 2>&1 ;;
    prccl) np=${arg%%/*}; bargs=${arg#*/}; [ "$bargs" = "$arg" ] && bargs=""
           (cd /tmp && HPCJOIN_SHARE_GPU=1 timeout -k 10 600 rocprofv3 --kernel-trace -d "$OUT/trace$n" -o run \
              --output-format csv -- python "$R/bench.py" --gpus $np ${bargs//,/ }) > "$log" 2>&1 ;;
    abbench) rc=0
             for i in 1 2; do
               (cd "$R/ab/base" && timeout -k 10 300 python -u bench.py $args > "$OUT/$n.base$i.log" 2>&1) || { rc=$?; break; }
               timeout -k 10 300 python -u bench.py $args > "$OUT/$n.new$i.log" 2>&1 || { rc=$?; break; }
             done
             echo "abbench rc=$rc" > "$log"; (exit $rc) ;;
    py) timeout -k 10 900 python -u $args > "$log" 2>&1 ;;
    epy) envs=${arg%%/*}; pargs=${arg#*/}
         timeout -k 10 900 env ${envs//,/ } python -u ${pargs//,/ } > "$log" 2>&1 ;;
    stats) (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/stats$n" -o run --output-format csv \
              -- python "$R/bench.py" $args) > "$log" 2>&1 ;;
    estats) envs=${arg%%/*}; bargs=${arg#*/}
            (cd /tmp && export ${envs//,/ } && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/stats$n" \
               -o run --output-format csv -- python "$R/bench.py" ${bargs//,/ }) > "$log" 2>&1 ;;
    pstats) (cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT/stats$n" -o run --output-format csv \
              -- python "$R/"$args) > "$log" 2>&1 ;;
    ppmc) ctrs=${arg%%/*}; sargs=${arg#*/}; (cd /tmp && timeout -s KILL 600 rocprofv3 --kernel-trace --pmc ${ctrs//,/ } \
              -d "$OUT/pmc$n" -o run --output-format csv -- python "$R/"${sargs//,/ }) > "$log" 2>&1 ;;
    pmc) ctrs=${arg%%/*}; bargs=${arg#*/}; (cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc ${ctrs//,/ } \
              -d "$OUT/pmc$n" -o run --output-format csv -- python "$R/bench.py" ${bargs//,/ }) > "$log" 2>&1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  tail -3 "$log"
  if [ $rc -ne 0 ]; then
    echo "[$n] $step failed rc=$rc"
    tail -40 "$log"
    exit $rc
  fi
done
echo done
