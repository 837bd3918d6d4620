"""allreducetopk_amd -- MI355X-native ARC-TopK gradient-compression comm hook.

Drop-in for the hot path of Aris-ma/AllreduceTopK: the DDP comm hooks in
``allreducetopk_amd.comm_hooks`` (same names, arguments, flags and state as the
reference's ``comm_hooks``) run their per-bucket codec as HIP kernels of
``lib/libarctopk.so`` (C ABI: ``include/arctopk.h``) with RCCL collectives.
"""
__version__ = "0.1.0"
