#!/bin/bash
# fp8 QKV / cross-Q dgrads: kernel + fp8 training tests, then C4 A/B
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -q --timeout 200 --timeout-method thread"
timeout -k 10 500 $T tests/test_kernels_gpu.py -k "attention" tests/test_prod_gpu.py::test_fp8_backward_building_blocks tests/test_prod_gpu.py::test_fp8_dgrad_training_tracks_bf16_dgrad tests/test_prod_gpu.py::test_fp8_training_reduces_loss_and_uses_fp8_kernels > gpurun_out/f8a_tests.log 2>&1
r=$?; tail -3 gpurun_out/f8a_tests.log; grep -h "^FAILED" gpurun_out/f8a_tests.log | head; [ $r -eq 0 ] || exit $r
timeout -k 10 600 python tools/ab_step.py c4 SMER_FP8_ATTN_DGRAD 0 1 --rounds=2 > gpurun_out/f8a_ab.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/f8a_ab.log | tail -2
