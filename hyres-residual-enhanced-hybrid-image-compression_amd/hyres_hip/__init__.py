"""hyres_hip — MI355X (gfx950) runtime for the HyRES residual-codec hot path.

libhyres_hip.so (csrc/*.hip, C-ABI in include/hyres_hip.h) + a thin Python layer: ctypes binding
(_lib), the NHWC op library with its reverse-mode tape (ops, entropy_ops, refine_ops), module classes
with reference-identical state_dict keys (layers), the RD loss (loss), the fused optimiser (optim) and
the data-parallel gradient reducer over RCCL (ddp)."""
__version__ = "0.1.0"
