"""igm_amd -- MI355X-native engine for the IGM (bonimba87/igm) hot path.

  igm_amd.astep    A-step: activation distances (ActivationDistanceStep.get_actdist)
  igm_amd.mstep    M-step: batched anneal + CG replacing the serial-LAMMPS kernel
  igm_amd._lib     ctypes binding of libigmhip.so (include/igm_hip.h)
"""
__version__ = '0.1.0'
