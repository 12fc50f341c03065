"""MI355X-native LightGCN propagation engine (drop-in for the reference's models/lightgcn.py path).

    engine   ctypes binding of liblgcn_engine.so (include/lgcn.h), CSR plan cache, autograd
    graph    host-side normalised-adjacency builder (main.py:282-336) + synthetic generators
    loss     bpr_loss_reg with the reference signature (main.py:366-402)
    dist     multi-GPU propagation (row partition + per-layer RCCL all-gather; feature split)
"""
__version__ = "0.1.0"
