"""config.debug=True forward (reference models/lightgcn.py:49-51 per-layer brand norms and
:62-78 cosine check, including its torch.manual_seed(42) side effect on the caller's RNG) against
fixtures produced by the reference itself (tests/golden/gen_golden.py debug): the printed lines,
the CPU generator's next draws after the forward, and the final embeddings (bitwise)."""
import contextlib
import io
import re

import numpy as np
import pytest
import torch

from conftest import Cfg, load_case
from gcn_recommendation_amd import graph
from util import sha1

CASES = ["debug_c1_brand", "debug_c1_brand_k0"]


def _run(z, dev):
    from models.lightgcn import LightGCN
    U, I, B, d, K = (int(z[k]) for k in ("U", "I", "B", "d", "K"))
    if dev.type == "cpu":
        idx = torch.from_numpy(np.vstack([z["adj_row"], z["adj_col"]]).astype(np.int64))
        adj = torch.sparse_coo_tensor(idx, torch.from_numpy(z["adj_val"]), (U + I + B,) * 2)
    else:
        adj = graph.build_norm_adj(z["train_user"], z["train_item"], U, I, B, z["ib_item"],
                                   z["ib_brand"], bool(z["use_brand"]), device=dev)
    torch.manual_seed(42)
    with contextlib.redirect_stdout(io.StringIO()):
        m = LightGCN(U, I, B, Cfg(d, K, debug=True)).to(dev)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        fu, fi, fb, _, _ = m(adj, use_brand=bool(z["use_brand"]))
    rng_after = torch.rand(8).numpy()
    final = torch.cat([fu, fi, fb]).detach().cpu().numpy()
    return buf.getvalue(), rng_after, final


def _numbers(text):
    return [(ln.split(":")[0], float(re.findall(r"[-+0-9.eE]+$", ln.strip())[0]))
            for ln in text.strip().splitlines()]


def _check(z, out, rng_after, final, tol):
    want = _numbers(str(z["stdout"]))
    got = _numbers(out)
    assert [k for k, _ in got] == [k for k, _ in want], out  # same lines, same order
    for (k, g), (_, w) in zip(got, want):
        assert abs(g - w) <= tol * max(1.0, abs(w)), (k, g, w)
    np.testing.assert_array_equal(rng_after, z["rng_after"])  # manual_seed(42) side effect
    assert sha1(final) == str(z["sha1/final"])


@pytest.mark.parametrize("name", CASES)
def test_debug_cpu_dispatch_matches_reference(name):
    """CPU adjacency: the drop-in runs the reference's own ATen ops — identical text."""
    z = load_case(name)
    out, rng_after, final = _run(z, torch.device("cpu"))
    assert out == str(z["stdout"])
    _check(z, out, rng_after, final, 0.0)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_debug_hip_path_matches_reference(gpu_device, name):
    """HIP path: layer outputs are bitwise the reference's, so the printed norms agree to the
    printed precision; the cosine check's dense matmul runs on the GPU (1e-5)."""
    z = load_case(name)
    out, rng_after, final = _run(z, gpu_device)
    _check(z, out, rng_after, final, 1e-5)
