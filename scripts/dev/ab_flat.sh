# wave-flattened bonds in the force kernel (IGM_POP_FLAT=2): parity checks under the variant library, then anneal A/B
# (125 structures, full protocol)
set -o pipefail
IGM_HIP_LIB=igm_amd/lib/ab/libigmhip_flatb7.so timeout -k 10 400 python -u -m pytest tests/test_mstep_paths_gpu.py tests/test_configDE_gpu.py -k "200kb and not stagewise" -x -v -rfE --tb=short --timeout 300 --timeout-method thread > gpurun_out/r06_flatb_pytest.log 2>&1
rc=$?; tail -12 gpurun_out/r06_flatb_pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=r06_flatb ARGS="--config C --nstruct 125" TLIM=200 VARIANTS=$'IGM_POP_X=0\nIGM_HIP_LIB=igm_amd/lib/ab/libigmhip_flatb7.so\nIGM_HIP_LIB=igm_amd/lib/ab/libigmhip_flatb6.so\nIGM_POP_X=0\nIGM_HIP_LIB=igm_amd/lib/ab/libigmhip_flatb7.so' bash scripts/gpu_variants.sh
