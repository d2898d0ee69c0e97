#!/bin/bash
# Vivaldi parity tests + default Vivaldi bench line
S=scripts/gpu_step.sh
bash $S pytest_viv 400 python -u -m pytest tests/test_vivaldi_gpu.py tests/test_codec_gpu.py -x -q --timeout 120 --timeout-method thread && \
bash $S bench_vivaldi 400 python -u bench.py --workload vivaldi --no-cpu-baseline
