#!/bin/bash
# One documented runner for GPU-box work (one `gpurun` call per invocation):
#
#   gpurun --timeout 1200 -- 'bash tools/gpu.sh full'            # -m gpu suite, smoke(), default bench line
#   gpurun -- 'bash tools/gpu.sh tests "<pytest -k expr>" [files]' # a subset of the GPU tests
#   gpurun -- 'bash tools/gpu.sh bench [bench.py args]'          # one bench line
#   gpurun -- 'bash tools/gpu.sh prof <tag>'                     # tools/profile_round.sh <tag>
#   gpurun -- 'bash tools/gpu.sh ab <c2|c4|c4bf16> ENV A B [--rounds=N]'  # train-step A/B of one switch
#   gpurun -- 'bash tools/gpu.sh kernels <gemm|attn|attn_c4|...> [lib ...]' # tools/bench_kernels.py per library
#   gpurun -- 'bash tools/gpu.sh py <script.py> [args]'          # any tools/ script under a 300 s limit
#
# A library argument `lib` names smer_music_generation_amd/_var/<lib>.so (built by
# tools/build_variant.sh); `tree` is the in-tree libsmer_hip.so.  Every GPU
# step has its own time limit and the steps are chained with && (a failed,
# aborted or timed-out step ends the call).  Logs go to gpurun_out/<sub>_*.log.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/smer_music_generation_amd/_var
PYT="python -u -m pytest --timeout 200 --timeout-method thread"
sub=${1:-full}; shift
libenv() { if [ "$1" = tree ]; then echo ""; else echo "SMER_HIP_LIB=$V/$1.so"; fi; }
case $sub in
  full)
    timeout -k 10 900 $PYT tests -m gpu -v > gpurun_out/full_gputest.log 2>&1; r=$?
    tail -3 gpurun_out/full_gputest.log; grep -h "^FAILED" gpurun_out/full_gputest.log | head -20
    [ $r -eq 0 ] || exit $r
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 || exit $?
    timeout -k 10 500 python bench.py "$@" > gpurun_out/full_bench.log 2>&1 || exit $?
    grep '^{' gpurun_out/full_bench.log | tail -1 | cut -c1-600
    ;;
  tests)
    k=$1; shift
    files=${@:-tests}
    timeout -k 10 900 $PYT -m gpu -v -k "$k" $files > gpurun_out/tests.log 2>&1; r=$?
    tail -3 gpurun_out/tests.log; grep -h "^FAILED" gpurun_out/tests.log | head -20
    exit $r
    ;;
  bench)
    timeout -k 10 500 python bench.py "$@" > gpurun_out/bench.log 2>&1 || exit $?
    grep '^{' gpurun_out/bench.log | tail -1 | cut -c1-800
    ;;
  prof)
    bash tools/profile_round.sh ${1:?tag} > gpurun_out/prof_$1.log 2>&1
    ;;
  ab)
    timeout -k 10 900 python tools/ab_step.py "$@" > gpurun_out/ab.log 2>&1 || exit $?
    grep -v amdgpu.ids gpurun_out/ab.log | tail -4
    ;;
  kernels)
    which=$1; shift
    for lib in ${@:-tree}; do
      env $(libenv $lib) timeout -k 10 300 python tools/bench_kernels.py $which > gpurun_out/kernels_${which}_$lib.log 2>&1 || exit $?
      echo "== $lib"; grep -v amdgpu.ids gpurun_out/kernels_${which}_$lib.log
    done
    ;;
  py)
    s=$1; shift
    timeout -k 10 300 python "$s" "$@" > gpurun_out/py_$(basename $s .py).log 2>&1; r=$?
    grep -v amdgpu.ids gpurun_out/py_$(basename $s .py).log | tail -40
    exit $r
    ;;
  *) echo "unknown subcommand $sub"; exit 2 ;;
esac
