#!/bin/bash
# One-group kernel traces (no kernel overlap) of the slack-sorted lists against IGM_POP_SLACK=0.
cd "$GRAFT_REPO_ROOT" || exit 1
NOPMC=1 TAG=kt_slk1 IGM_POP_GROUPS=1 SCALE=0.02 bash scripts/gpu_prof1000.sh && \
NOPMC=1 TAG=kt_slk0 IGM_POP_GROUPS=1 SCALE=0.02 IGM_HIP_LIB=igm_amd/lib/ab/libigmhip_slk0.so bash scripts/gpu_prof1000.sh
