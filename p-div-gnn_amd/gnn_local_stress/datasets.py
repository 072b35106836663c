"""``gnn_local_stress.datasets`` subset: ``NodeType`` (reference datasets.py:33-36) and
the graph helpers of the input format, on synthetic meshes (pdg.meshgen).

The reference's ``MeshStressFieldDatasetInMemory`` reads gmsh/fedoo ``.vtk`` +
``.npz`` files through pyvista (absent here; out of scope)."""
from enum import IntEnum


class NodeType(IntEnum):
    INTERNAL_BOUNDARY = -1
    INTERNAL = 0
    EXTERNAL_BOUNDARY = 1
