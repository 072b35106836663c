"""MI355X drop-in for the reference package ``gnn_local_stress`` (hot path only).

models (EncodeProcessDecode & co.), data_utils, datasets.NodeType and the
training losses (reference: scripts/gnn_train.py:41-92) are provided; the FEM
dataset/mesh conversion modules are out of scope."""
