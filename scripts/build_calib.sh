#!/bin/bash
# build the counter-calibration microbenchmark (scripts/gather_calib.hip) in-tree for gfx950
set -e
cd "$(dirname "$0")/.."
mkdir -p igm_amd/lib/calib
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -o igm_amd/lib/calib/gather_calib scripts/gather_calib.hip
echo built igm_amd/lib/calib/gather_calib
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -o igm_amd/lib/calib/gather_rate scripts/gather_rate.hip
echo built igm_amd/lib/calib/gather_rate
