#!/bin/bash
# Builds and runs the PMC calibration (three rocprofv3 passes), then prints the ratios.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
D=gpurun_out/pmc_calib; mkdir -p $D
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 experiments/pmc_calib.hip -o $D/pmc_calib || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $D/trace -o run -- $D/pmc_calib > $D/calib.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- $D/pmc_calib > $D/fetch.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- $D/pmc_calib > $D/write.log 2>&1 || exit $?
python3 experiments/pmc_calib.py $D | tee $D/summary.txt
