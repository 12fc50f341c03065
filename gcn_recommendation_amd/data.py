"""On-disk formats of the reference: the processed-data directory written by
dataset/*/prepare_data.py — train.parquet / test.parquet (user_idx, item_idx), item_brand.parquet
(item_idx, brand_idx; several rows per item for the multi-category scripts), stats.json
(num_users, num_items, num_brands) and item_embeddings.npy ([num_items x C] fp32, zero rows for
items without metadata) — loaded into the reference's 8-tuple (main.py:172-347), with Â built on
the HIP device (graph.build_norm_adj_device) and its CSR plan already attached.
"""
import json
import os

import numpy as np
import pandas as pd
import torch

from . import graph


def load_preprocessed_data(data_dir, device, use_brand=True, debug=False, verbose=True):
    """Same inputs, same split and same return tuple as main.py:172-347:
    (train_df, val_df, test_df, num_users, num_items, num_brands, norm_adj_tensor, item_brand_df).
    """
    stats_path = os.path.join(data_dir, "stats.json")
    if not os.path.exists(stats_path):
        raise FileNotFoundError(f"Stats file not found in '{data_dir}'. Please run "
                                f"'prepare_data.py' first.")
    all_train_df = pd.read_parquet(os.path.join(data_dir, "train.parquet"))
    test_df = pd.read_parquet(os.path.join(data_dir, "test.parquet"))
    item_brand_df = pd.read_parquet(os.path.join(data_dir, "item_brand.parquet"))
    if debug:  # main.py:191-198: 1% of the users, drawn from numpy's global RNG
        unique_users = all_train_df["user_idx"].unique()
        sample_size = max(1, int(len(unique_users) * 0.01))
        sample_users = np.random.choice(unique_users, size=sample_size, replace=False)
        all_train_df = all_train_df[all_train_df["user_idx"].isin(sample_users)]
        test_df = test_df[test_df["user_idx"].isin(sample_users)]
    # main.py:201-203 verbatim: groupby(user).rank(method="first", ascending=False) over the
    # constant user column ranks a user's rows by appearance, so rank 1 — the validation row —
    # is the user's FIRST row in file order (tests/test_data_loader.py pins this)
    all_train_df = all_train_df.copy()
    all_train_df["rank"] = all_train_df.groupby("user_idx")["user_idx"].rank(method="first",
                                                                           ascending=False)
    val_df = all_train_df[all_train_df["rank"] == 1].copy()
    train_df = all_train_df[all_train_df["rank"] > 1].copy()
    with open(stats_path) as f:
        st = json.load(f)
    U, I, B = st["num_users"], st["num_items"], st["num_brands"]
    dev = torch.device(device)
    args = (train_df["user_idx"].to_numpy(), train_df["item_idx"].to_numpy(), U, I, B,
            item_brand_df["item_idx"].to_numpy(), item_brand_df["brand_idx"].to_numpy(),
            use_brand)
    if dev.type == "cuda":
        adj = graph.build_norm_adj_device(*args, device=dev)
    else:
        adj = graph.build_norm_adj(*args, device=dev)
    if verbose:
        print(f"[lgcn] {data_dir}: users {U:,} items {I:,} brands {B:,} | train {len(train_df):,} "
              f"val {len(val_df):,} test {len(test_df):,} | nnz(Â) {adj._nnz():,} "
              f"({'with' if use_brand else 'no'} brand edges) on {dev}")
    return train_df, val_df, test_df, U, I, B, adj, item_brand_df


def load_item_embeddings(data_dir):
    """item_embeddings.npy (amazon_books_emb/prepare_data.py:141-150) without unpickling."""
    return np.load(os.path.join(data_dir, "item_embeddings.npy"), allow_pickle=False)
