"""Minimal HIP-graph capture of nested stream forks (torch only): origin -> A -> B, B joined
into A and A into origin (variant 'nested'); or B also joined into origin ('direct'); or B first waits on the origin ('pre')."""
import sys

import torch

dev = torch.device("cuda:0")
x = torch.ones(1 << 20, device=dev)
A, B = torch.cuda.Stream(), torch.cuda.Stream()
g = torch.cuda.CUDAGraph()
mode = sys.argv[1]
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    with torch.cuda.graph(g):
        o = torch.cuda.current_stream()
        A.wait_stream(o)
        if mode == "pre":  # B enters the capture from the origin first
            B.wait_stream(o)
        with torch.cuda.stream(A):
            y = x * 2
            B.wait_stream(A)
            with torch.cuda.stream(B):
                z = x * 3
            A.wait_stream(B)
            w = y + z
        o.wait_stream(A)
        if mode == "direct":
            o.wait_stream(B)
        out = w * 1
g.replay()
torch.cuda.synchronize()
print(mode, "ok", float(out[0]))
