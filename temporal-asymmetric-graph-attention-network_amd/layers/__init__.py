"""Hot-path layers (mirror of src/tagan/layers/__init__.py)."""
from .geometric_attention import GeometricAttention, GeometricAttentionLayer, DistanceMetric  # noqa: F401
from .temporal_propagation import TemporalPropagation  # noqa: F401
from .temporal_attention import TemporalAttention, AsymmetricTemporalAttention, TimeEncoding  # noqa: F401
from .classification import ClassificationModule  # noqa: F401
from .graph_attention import TAGANGraphAttention  # noqa: F401
