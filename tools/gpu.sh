#!/bin/bash
# One parameterised GPU-box pass (replaces the per-experiment tools/gpu_r02*.sh one-shots).
#
#   bash tools/gpu.sh <tag> <step> [<step> ...]
#
# Outputs go to gpurun_out/<tag>/.  Every GPU step runs under its own time limit and the pass stops at the
# first failing step (set -e): nothing else touches the GPU after a fault, abort or timeout.
# Steps:
#   tests[=<pytest -k expr>]   GPU suite (or the selected tests), -s output kept (printed errors)
#   file=<test file(s)>        the GPU tests of these files
#   smoke                      __graft_entry__.smoke()
#   c2 | c2cpu                 C2 bench line (c2cpu: with the CPU baseline)
#   c2at=<dir>                 C2 bench line of the tree copy in <dir> (A/B arm)
#   c3 | c4 | c4b8 | c5        C3 batch 8, C4 KITTI 64-beam (batch 1 / 8), C5 10-seed ensemble bench lines
#   c4at=<dir> | c5at=<dir>    the C4 / C5 bench line of the tree copy in <dir> (A/B arm)
#   trace                      rocprofv3 --kernel-trace --stats of a short C2 bench
#   trace3                     the same for C3 (batch 8)
#   calltrace                  kernel trace of 4 C2 calls, itemised outside the step graphs (tools/call_timeline.py)
#   pmc | pmc8                 FETCH_SIZE, WRITE_SIZE, MFMA-busy passes over the conv kernels (eager C2 / C3, 4 steps)
#   breakdown[=<batch>]        per-shape conv breakdown of one guided step (tools/conv_breakdown.py)
#   stepprof                   per-shape conv time inside the graph-replayed step (tools/step_profile.py)
#   pmcstep                    FETCH_SIZE / WRITE_SIZE / MFMA-busy passes over that same step (tools/pmc_step.py)
#   py=<script args>           any repo python script (e.g. py=tools/gemm_one.py --m 6912)
#   tune=<workloads>           time the shapes missing from the committed table (DC_TUNE_COLD=2), e.g. tune=c2:1,c2:8
#   tunefresh=<workloads>      the same over every shape of the workloads (--fresh: the committed table ignored)
#   usetuned                   use that table (copied over the box's tree copy) for the following steps
#   c2env=<K>=<V>[,<K>=<V>]    C2 bench line with these environment variables (an A/B arm of an opt-in switch)
#   c3env=<K>=<V>[,<K>=<V>]    the same for C3 (batch 8)
set -e
tag=${1:?tag}
shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  case "$step" in
    tests)
      timeout -k 10 1500 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
        > "$out/gputest.log" 2>&1 ;;
    tests=*)
      timeout -k 10 1200 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread -k "${step#tests=}" \
        > "$out/gputest_$n.log" 2>&1 ;;
    file=*)
      # shellcheck disable=SC2086
      timeout -k 10 1200 python -u -m pytest ${step#file=} -m gpu -v -s --timeout 600 --timeout-method thread \
        > "$out/gputest_$n.log" 2>&1 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 ;;
    c2)
      timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$out/bench_c2.json" 2> "$out/bench_c2.err"
      cp "$out/bench_c2.json" "$out/bench_c2_$n.json" ;;
    c2at=*)
      # the C2 bench line of another tree (an A/B arm: a full copy of a tree with its built library, e.g. ab/old)
      d=${step#c2at=}
      (cd "$d" && timeout -k 10 400 python -u bench.py --no-cpu-baseline) > "$out/bench_c2_$n.json" 2> "$out/bench_c2_$n.err" ;;
    c4at=*)
      d=${step#c4at=}
      (cd "$d" && timeout -k 10 300 python -u bench.py --height 352 --width 1216 --pattern beams --no-cpu-baseline) \
        > "$out/bench_c4_$n.json" 2> "$out/bench_c4_$n.err" ;;
    c5at=*)
      d=${step#c5at=}
      (cd "$d" && timeout -k 10 400 python -u bench.py --height 900 --width 1600 --points 3000 --seeds 10 --steps 2 \
        --warmup 1 --no-cpu-baseline) > "$out/bench_c5_$n.json" 2> "$out/bench_c5_$n.err" ;;
    c2cpu)
      timeout -k 10 600 python -u bench.py > "$out/bench_c2.json" 2> "$out/bench_c2.err" ;;
    c3)
      timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline \
        > "$out/bench_c3_b8.json" 2> "$out/bench_c3_b8.err" ;;
    c4)
      timeout -k 10 300 python -u bench.py --height 352 --width 1216 --pattern beams --no-cpu-baseline \
        > "$out/bench_c4.json" 2> "$out/bench_c4.err"
      cp "$out/bench_c4.json" "$out/bench_c4_$n.json" ;;
    c4b8)
      timeout -k 10 300 python -u bench.py --height 352 --width 1216 --pattern beams --batch 8 --steps 2 --warmup 1 \
        --no-cpu-baseline > "$out/bench_c4_b8.json" 2> "$out/bench_c4_b8.err" ;;
    c5)
      timeout -k 10 400 python -u bench.py --height 900 --width 1600 --points 3000 --seeds 10 --steps 2 --warmup 1 \
        --no-cpu-baseline > "$out/bench_c5.json" 2> "$out/bench_c5.err"
      cp "$out/bench_c5.json" "$out/bench_c5_$n.json" ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$out/trace_bench.json" 2> "$out/trace.err" ;;
    calltrace)
      # per-call time outside the step graphs (tools/call_timeline.py): 4 calls, 3 stretches between them
      timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/calltrace" -o run --output-format csv -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$out/calltrace_bench.json" 2> "$out/calltrace.err"
      python3 tools/call_timeline.py "$out/calltrace/run_kernel_trace.csv" > "$out/call_timeline.txt" 2>&1 ;;
    trace3)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace3" -o run --output-format csv -- \
        python3 bench.py --batch 8 --steps 1 --warmup 1 --no-cpu-baseline > "$out/trace3_bench.json" 2> "$out/trace3.err" ;;
    pmc|pmc8)
      # FETCH_SIZE, WRITE_SIZE and the MFMA-busy pass over the conv kernels (im2col, halo and skinny), eager step, 4 denoise
      # steps; each pass its own run (rocprofv3 does not split counters over passes)
      b=1; [ "$step" = pmc8 ] && b=8
      for pass in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE:mfma"; do
        # shellcheck disable=SC2086
        timeout -s KILL 180 rocprofv3 --pmc ${pass%%:*} --kernel-include-regex "conv_(gemm|halo|skinny)_kernel" \
          -d "$out/pmc${b}_${pass##*:}" -o run --output-format csv -- python3 bench.py --no-graph --steps 1 --warmup 0 \
          --no-cpu-baseline --denoise-steps 4 --batch $b > "$out/pmc${b}_${pass##*:}.json" 2> "$out/pmc${b}_${pass##*:}.err"
      done ;;
    stepprof)
      timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/steptrace" -o run --output-format csv -- \
        python3 tools/step_profile.py --out "$out/descs.json" > "$out/stepprof.log" 2>&1
      python3 tools/step_profile.py --trace "$out/steptrace/run_kernel_trace.csv" --descs "$out/descs.json" \
        > "$out/step_shapes.txt" 2>&1 ;;
    pmcstep)
      # PMC passes over the graph-replayed step (one counter set per pass), then the per-step / per-launch record
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$out/pmcf" -o run --output-format csv -- \
        python3 tools/step_profile.py --out "$out/descs.json" > "$out/pmcf.log" 2>&1
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$out/pmcw" -o run --output-format csv -- \
        python3 tools/step_profile.py --out "$out/descs.json" > "$out/pmcw.log" 2>&1
      timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$out/pmcm" -o run \
        --output-format csv -- python3 tools/step_profile.py --out "$out/descs.json" > "$out/pmcm.log" 2>&1
      python3 tools/pmc_step.py "$out/pmcf/run_counter_collection.csv" "$out/pmcw/run_counter_collection.csv" \
        "$out/pmcm/run_counter_collection.csv" "$out/descs.json" "$out/pmc_step.json" > "$out/pmc_step.log" 2>&1 ;;
    breakdown)
      timeout -k 10 300 python -u tools/conv_breakdown.py > "$out/conv_breakdown.txt" 2> "$out/conv_breakdown.err" ;;
    breakdown=*)
      timeout -k 10 300 python -u tools/conv_breakdown.py --batch "${step#breakdown=}" \
        > "$out/conv_breakdown_b${step#breakdown=}.txt" 2> "$out/conv_breakdown.err" ;;
    py=*)
      # shellcheck disable=SC2086
      timeout -k 10 600 python -u ${step#py=} > "$out/py_$n.txt" 2> "$out/py_$n.err" ;;
    tune=*)
      # shellcheck disable=SC2046
      DC_TUNE_COLD=2 timeout -k 10 900 python -u tools/tune_gemm.py --workloads $(echo "${step#tune=}" | tr , ' ') \
        --out "$out/tuned_gfx950.json" > "$out/tune.log" 2>&1 ;;
    tunefresh=*)
      # shellcheck disable=SC2046
      DC_TUNE_COLD=2 timeout -k 10 1100 python -u tools/tune_gemm.py --fresh --workloads $(echo "${step#tunefresh=}" | tr , ' ') \
        --out "$out/tuned_gfx950.json" > "$out/tune.log" 2>&1 ;;
    usetuned)
      cp "$out/tuned_gfx950.json" depth_completion_amd/tuned_gfx950.json ;;
    c2env=*)
      # shellcheck disable=SC2046
      env $(echo "${step#c2env=}" | tr , ' ') timeout -k 10 400 python -u bench.py --no-cpu-baseline \
        > "$out/bench_c2_$n.json" 2> "$out/bench_c2_$n.err" ;;
    c3env=*)
      # shellcheck disable=SC2046
      env $(echo "${step#c3env=}" | tr , ' ') timeout -k 10 400 python -u bench.py --batch 8 --steps 2 --warmup 1 \
        --no-cpu-baseline > "$out/bench_c3_$n.json" 2> "$out/bench_c3_$n.err" ;;
    *)
      echo "unknown step $step" >&2
      exit 2 ;;
  esac
  echo "[$tag] step $n ($step) done"
done
echo "[$tag] all done"
