"""Drop-in `models.lightgcn_fusion.LightGCN_Fusion` (reference models/lightgcn_fusion.py:5-64).

Same constructor (raises without pretrained content embeddings), module registration and RNG
order (user, item_id, brand embeddings, fusion Linear, then four xavier inits), buffer
`item_content_embedding`, and 5-tuple. The item pre-fusion `leaky_relu(Linear([id ‖ content]))`
(lightgcn_fusion.py:45-49) runs as one engine kernel on a HIP device (no concatenation, MFMA GEMM
with bias + leaky_relu fused, gcn_recommendation_amd.fusion); the K-layer
propagation + mean (lightgcn_fusion.py:55-59) runs in the MI355X engine, reading
E0 = [user | fused_item | brand] as three segments.
"""
import torch
import torch.nn as nn

from gcn_recommendation_amd import engine, fusion


class LightGCN_Fusion(nn.Module):
    def __init__(self, num_users, num_items, num_brands, config, pretrained_item_emb=None):
        super(LightGCN_Fusion, self).__init__()
        self.num_users = num_users
        self.num_items = num_items
        self.num_brands = num_brands
        self.embedding_dim = config.embedding_dim
        self.n_layers = config.n_layers
        if pretrained_item_emb is None:
            raise ValueError("LightGCN_Fusion model requires pretrained item embeddings.")
        content_emb_dim = pretrained_item_emb.shape[1]
        self.user_embedding = nn.Embedding(num_users, self.embedding_dim)
        self.item_id_embedding = nn.Embedding(num_items, self.embedding_dim)
        self.brand_embedding = nn.Embedding(num_brands, self.embedding_dim)
        self.register_buffer('item_content_embedding', torch.FloatTensor(pretrained_item_emb))
        self.item_fusion_layer = nn.Linear(self.embedding_dim + content_emb_dim, self.embedding_dim)
        nn.init.xavier_uniform_(self.user_embedding.weight)
        nn.init.xavier_uniform_(self.item_id_embedding.weight)
        nn.init.xavier_uniform_(self.brand_embedding.weight)
        nn.init.xavier_uniform_(self.item_fusion_layer.weight)
        self._graph_adj = None

    def fused_item_embedding(self):
        # lightgcn_fusion.py:45-49; on a HIP device one engine kernel (gcn_recommendation_amd.fusion)
        return fusion.fused_item_embedding(self.item_id_embedding.weight,
                                           self.item_content_embedding, self.item_fusion_layer)

    def forward(self, adj_mat, use_brand=True):
        user_emb_0 = self.user_embedding.weight
        item_id_emb_0 = self.item_id_embedding.weight
        brand_emb_0 = self.brand_embedding.weight
        fused_item_emb_0 = self.fused_item_embedding()
        segments = [user_emb_0, fused_item_emb_0, brand_emb_0]
        if adj_mat.device.type == "cuda":
            # user_emb_0 as the engine's alias: its gradient joins the propagation's inside the
            # backward (engine.PropagateFunction, e0_outputs)
            final_user_emb, final_item_emb, final_brand_emb, user_emb_0 = engine.propagate_blocks(
                adj_mat, segments, self.n_layers, e0_outputs=1)
        else:  # CPU adjacency: the reference's ATen path (lightgcn_fusion.py:52-59)
            ego = torch.cat(segments, dim=0)
            all_embeddings = [ego]
            for _ in range(self.n_layers):
                ego = torch.sparse.mm(adj_mat, ego)
                all_embeddings.append(ego)
            final_embeddings = torch.mean(torch.stack(all_embeddings, dim=0), dim=0)
            final_user_emb, final_item_emb, final_brand_emb = torch.split(
                final_embeddings, [self.num_users, self.num_items, self.num_brands])
        return final_user_emb, final_item_emb, final_brand_emb, user_emb_0, item_id_emb_0

    def set_graph(self, adj_mat):
        self._graph_adj = adj_mat
        return self

    def computer(self, adj_mat=None):
        adj = adj_mat if adj_mat is not None else self._graph_adj
        if adj is None:
            raise ValueError("computer() needs adj_mat (or set_graph(adj_mat) first)")
        fu, fi, _, _, _ = self.forward(adj)
        return fu, fi
