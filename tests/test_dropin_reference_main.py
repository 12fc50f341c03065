"""End-to-end drop-in: the reference's own main.py (unchanged, imported from /root/reference —
only present in the build container, so this test skips elsewhere) trains, validates,
checkpoints and tests with THIS repo's models/ plugins, via tools/run_reference_main.py."""
import json
import os
import subprocess
import sys

import numpy as np
import pandas as pd
import pytest

from conftest import ROOT

REF_MAIN = "/root/reference/main.py"


@pytest.mark.skipif(not os.path.exists(REF_MAIN), reason="reference repo not mounted")
@pytest.mark.parametrize("model,extra", [("LightGCN", []),
                                         ("LightGCN_Fusion", ["--use_pretrained_emb"])])
def test_reference_main_train_then_test(tmp_path, model, extra):
    d = tmp_path / "dataset" / "steam_emb" / "processed_data_16"
    d.mkdir(parents=True)
    rng = np.random.default_rng(0)
    U, I, B, E = 300, 200, 20, 4000
    pd.DataFrame({"user_idx": rng.integers(0, U, E), "item_idx": rng.integers(0, I, E)}) \
        .to_parquet(d / "train.parquet")
    pd.DataFrame({"user_idx": np.arange(U), "item_idx": rng.integers(0, I, U)}) \
        .to_parquet(d / "test.parquet")
    pd.DataFrame({"item_idx": np.arange(I), "brand_idx": rng.integers(0, B, I)}) \
        .to_parquet(d / "item_brand.parquet")
    json.dump({"num_users": U, "num_items": I, "num_brands": B}, open(d / "stats.json", "w"))
    np.save(d / "item_embeddings.npy", rng.standard_normal((I, 64)).astype(np.float32))
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", MPLBACKEND="Agg")
    runner = os.path.join(ROOT, "tools", "run_reference_main.py")
    tr = subprocess.run([sys.executable, runner, REF_MAIN, "train", "--model_name", model,
                         "--epochs", "5"] + extra, cwd=tmp_path, env=env, capture_output=True,
                        text=True, timeout=600)
    assert tr.returncode == 0, tr.stderr[-2000:]
    assert "Val Recall@20" in tr.stdout and "New best model saved" in tr.stdout
    te = subprocess.run([sys.executable, runner, REF_MAIN, "test", "--model_name", model] + extra,
                        cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert te.returncode == 0, te.stderr[-2000:]
    assert "Recall@20:" in te.stdout and "Model loaded from" in te.stdout
