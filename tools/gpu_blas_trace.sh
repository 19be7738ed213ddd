#!/bin/bash
# kernel names / durations of the rocBLAS bar (which macro tile rocBLAS picks for each shape)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/blas_trace
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/blas_trace -o run -- ./tools/blas_bar > gpurun_out/blas_trace/log 2>&1 && echo "blas trace ok"
