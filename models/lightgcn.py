"""Drop-in `models.lightgcn.LightGCN` for the reference's plugin loader (main.py:42-50).

`importlib.import_module("models.lightgcn")` + `getattr(mod, "LightGCN")` resolves this class
unchanged. Constructor, RNG draw order, parameter order, state_dict keys, forward signature and
the 5-tuple it returns are those of the reference (models/lightgcn.py:4-81). The propagation
(lightgcn.py:37-54) runs on a HIP device in the MI355X engine (gcn_recommendation_amd.engine:
hand-written gfx950 CSR-SpMM kernels behind a C ABI, fused layer mean, custom autograd backward).
A CPU adjacency runs the reference's own ATen ops (device dispatch, as the reference does on a
CPU-only host — never a fallback for a HIP tensor: the engine raises if it cannot run).
"""
import torch
import torch.nn as nn

from gcn_recommendation_amd import engine


class LightGCN(nn.Module):
    def __init__(self, num_users, num_items, num_brands, config, pretrained_item_emb=None):
        super(LightGCN, self).__init__()
        self.num_users = num_users
        self.num_items = num_items
        self.num_brands = num_brands
        self.embedding_dim = config.embedding_dim
        self.n_layers = config.n_layers
        self.debug = config.debug

        # registration and RNG order as lightgcn.py:15-31: N(user), N(brand), [N(item)],
        # xavier(item), xavier(user), xavier(brand)
        self.user_embedding = nn.Embedding(num_users, self.embedding_dim)
        self.brand_embedding = nn.Embedding(num_brands, self.embedding_dim)
        if pretrained_item_emb is not None:
            print("INFO: Initializing item embeddings from pretrained file.")
            if pretrained_item_emb.shape[1] != self.embedding_dim:
                raise ValueError(f"Pretrained embedding dim ({pretrained_item_emb.shape[1]}) does "
                                 f"not match model embedding dim ({self.embedding_dim}).")
            self.item_embedding = nn.Embedding.from_pretrained(
                torch.FloatTensor(pretrained_item_emb), freeze=False)
        else:
            print("INFO: Randomly initializing item embeddings.")
            self.item_embedding = nn.Embedding(num_items, self.embedding_dim)
            nn.init.xavier_uniform_(self.item_embedding.weight)
        nn.init.xavier_uniform_(self.user_embedding.weight)
        nn.init.xavier_uniform_(self.brand_embedding.weight)
        self.final_brand_emb = None
        self._graph_adj = None

    # -- propagation ------------------------------------------------------------------------
    def _propagate(self, adj_mat, segments):
        """(final_user, final_item, final_brand) blocks, then the user and item ego tables: on a
        HIP device the engine's aliases of them (their gradients join the propagation's inside
        its backward — engine.PropagateFunction), on a CPU adjacency the weights themselves."""
        if adj_mat.device.type == "cuda":
            final = engine.propagate_blocks(adj_mat, segments, self.n_layers, e0_outputs=2)
            if self.debug and self.n_layers > 0:  # lightgcn.py:44-51 prints once per layer
                with torch.no_grad():
                    _, layers = engine.propagate_forward(
                        engine.graph_from_coo(adj_mat, engine.segment_sides(segments)),
                        [s.detach() for s in segments],
                        self.n_layers, return_layers=True)
                    off = self.num_users + self.num_items
                    for i, e in enumerate(layers + [None]):
                        if e is None:  # E_K is folded into the mean; recompute it for the print
                            e = self._last_layer(adj_mat, layers, segments)
                        print(f"Layer {i + 1} brand embedding L2 norm: {e[off:].norm(2).item():.6f}")
            return final
        # CPU adjacency: the reference's ATen path (lightgcn.py:40-54)
        ego = torch.cat(segments, dim=0)
        all_embeddings = [ego]
        for i in range(self.n_layers):
            ego = torch.sparse.mm(adj_mat, ego)
            all_embeddings.append(ego)
            if self.debug:
                brand_emb_i = ego[self.num_users + self.num_items:]
                print(f"Layer {i + 1} brand embedding L2 norm: {brand_emb_i.norm(2).item():.6f}")
        final = torch.mean(torch.stack(all_embeddings, dim=0), dim=0)
        return torch.split(final, [self.num_users, self.num_items, self.num_brands]) + \
            (segments[0], segments[1])

    def _last_layer(self, adj_mat, layers, segments):
        g = engine.graph_from_coo(adj_mat, engine.segment_sides(segments))
        x = layers[-1] if layers else torch.cat([s.detach() for s in segments], 0)
        y = torch.empty_like(x)
        return engine.spmm_layer(g, [x], y, x.shape[1], engine._epilogue(engine.LGCN_EPI_STORE),
                                 engine.hub_threshold_from_env())

    def forward(self, adj_mat, use_brand=True):
        # use_brand is accepted and ignored, exactly as lightgcn.py:35 (Â decides)
        user_emb_0 = self.user_embedding.weight
        item_emb_0 = self.item_embedding.weight
        brand_emb_0 = self.brand_embedding.weight
        final_user_emb, final_item_emb, final_brand_emb, user_emb_0, item_emb_0 = \
            self._propagate(adj_mat, [user_emb_0, item_emb_0, brand_emb_0])
        if self.debug:
            self._debug_cosine(adj_mat, final_item_emb, user_emb_0, item_emb_0)
        return final_user_emb, final_item_emb, final_brand_emb, user_emb_0, item_emb_0

    def _debug_cosine(self, adj_mat, final_item_emb, user_emb_0, item_emb_0):
        """lightgcn.py:62-78 diagnostics (dense, debug-only; identical semantics)."""
        torch.manual_seed(42)
        random_item_idx = torch.randint(0, self.num_items, (100,)).to(user_emb_0.device)
        item_emb_with_brand = final_item_emb[random_item_idx]
        adj_dense = adj_mat.to_dense()
        nui = self.num_users + self.num_items
        adj_user_item = adj_dense[:nui, :nui]
        ego_no_brand = torch.matmul(adj_user_item, torch.cat([user_emb_0, item_emb_0], dim=0))
        item_emb_no_brand = ego_no_brand[self.num_users:nui][random_item_idx]
        item_emb_no_brand = item_emb_0[random_item_idx] + item_emb_no_brand
        cos_sim = torch.nn.functional.cosine_similarity(
            item_emb_with_brand, item_emb_no_brand, dim=1).mean()
        print(f"Average cos similarity (item emb with/without brand): {cos_sim.item():.6f}")

    # -- LightGCN-style accessor (north_star "computer()") --------------------------------------
    def set_graph(self, adj_mat):
        self._graph_adj = adj_mat
        return self

    def computer(self, adj_mat=None):
        """(final_user [U,d], final_item [I,d]) — the propagated embeddings, as LightGCN's
        computer(). Uses `adj_mat` or the adjacency given to set_graph()."""
        adj = adj_mat if adj_mat is not None else self._graph_adj
        if adj is None:
            raise ValueError("computer() needs adj_mat (or set_graph(adj_mat) first)")
        fu, fi, fb, _, _ = self.forward(adj)
        self.final_brand_emb = fb
        return fu, fi
