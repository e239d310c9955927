"""TAGANConfig — same field names, defaults and validation as src/tagan/utils/config.py:14-350.

Build-only knobs (none needed on the hot path yet) stay out of this class so a
reference config dict / JSON file round-trips unchanged.  ``device`` keeps the
reference's 'cpu' | 'cuda' vocabulary; on ROCm 'cuda' is the HIP device.
"""
import json
import os
from typing import Any, Dict

import torch


class TAGANConfig:
    def __init__(self, hidden_dim: int = 64, num_layers: int = 2, num_heads: int = 4,
                 temporal_attention_dim: int = 64, node_feature_dim: int = 16, edge_feature_dim: int = 0,
                 output_dim: int = 2, learning_rate: float = 0.001, weight_decay: float = 1e-5,
                 dropout: float = 0.1, memory_decay_factor: float = 0.8, max_inactivity: int = 5,
                 gradient_clip_val: float = 1.0, use_layer_norm: bool = True, edge_importance: bool = True,
                 gru_bias: bool = True, leaky_relu_slope: float = 0.2, use_edge_features: bool = False,
                 concat_heads: bool = True, learnable_distance: bool = False, time_aware: bool = True,
                 bidirectional: bool = False, use_skip_connection: bool = True, use_gating: bool = True,
                 temporal_window_size: int = 3, aggregation_method: str = "mean", use_residual: bool = True,
                 causal_attention: bool = False, asymmetric_temporal_bias: bool = True, window_size: int = 5,
                 loss_type: str = "ce", focal_alpha: float = 0.25, focal_gamma: float = 2.0, num_epochs: int = 50,
                 device: str = "cuda" if torch.cuda.is_available() else "cpu"):
        self.hidden_dim = hidden_dim
        self.num_layers = num_layers
        self.num_heads = num_heads
        self.temporal_attention_dim = temporal_attention_dim
        self.node_feature_dim = node_feature_dim
        self.edge_feature_dim = edge_feature_dim if use_edge_features else 0   # config.py:145
        self.output_dim = output_dim
        self.learning_rate = learning_rate
        self.weight_decay = weight_decay
        self.dropout = dropout
        self.memory_decay_factor = memory_decay_factor
        self.max_inactivity = max_inactivity
        self.gradient_clip_val = gradient_clip_val
        self.num_epochs = num_epochs
        self.use_layer_norm = use_layer_norm
        self.edge_importance = edge_importance
        self.gru_bias = gru_bias
        self.leaky_relu_slope = leaky_relu_slope
        self.use_edge_features = use_edge_features
        self.concat_heads = concat_heads
        self.learnable_distance = learnable_distance
        self.time_aware = time_aware
        self.bidirectional = bidirectional
        self.use_skip_connection = use_skip_connection
        self.use_gating = use_gating
        self.temporal_window_size = temporal_window_size
        self.aggregation_method = aggregation_method
        self.use_residual = use_residual
        self.causal_attention = causal_attention
        self.asymmetric_temporal_bias = asymmetric_temporal_bias
        self.window_size = window_size
        self.loss_type = loss_type
        self.focal_alpha = focal_alpha
        self.focal_gamma = focal_gamma
        self.device = device
        self.validate()

    def validate(self):
        def need(cond, msg):
            if not cond:
                raise ValueError(msg)
        need(self.hidden_dim > 0, f"Hidden dimension must be positive, got {self.hidden_dim}")
        need(self.num_layers > 0, f"Number of layers must be positive, got {self.num_layers}")
        need(self.num_heads > 0, f"Number of heads must be positive, got {self.num_heads}")
        need(self.temporal_attention_dim > 0,
             f"Temporal attention dimension must be positive, got {self.temporal_attention_dim}")
        need(self.node_feature_dim > 0, f"Node feature dimension must be positive, got {self.node_feature_dim}")
        need(self.edge_feature_dim >= 0, f"Edge feature dimension must be non-negative, got {self.edge_feature_dim}")
        need(self.output_dim > 0, f"Output dimension must be positive, got {self.output_dim}")
        need(self.learning_rate > 0, f"Learning rate must be positive, got {self.learning_rate}")
        need(self.weight_decay >= 0, f"Weight decay must be non-negative, got {self.weight_decay}")
        need(0 <= self.dropout < 1, f"Dropout must be in [0, 1), got {self.dropout}")
        need(0 < self.memory_decay_factor <= 1,
             f"Memory decay factor must be in (0, 1], got {self.memory_decay_factor}")
        need(self.max_inactivity > 0, f"Maximum inactivity must be positive, got {self.max_inactivity}")
        need(self.gradient_clip_val >= 0, f"Gradient clip value must be non-negative, got {self.gradient_clip_val}")
        need(self.leaky_relu_slope > 0, f"LeakyReLU slope must be positive, got {self.leaky_relu_slope}")
        valid = ["ce", "bce", "mse", "focal"]
        need(self.loss_type in valid, f"Loss type must be one of {valid}, got {self.loss_type}")
        need(0 < self.focal_alpha < 1, f"Focal alpha must be in (0, 1), got {self.focal_alpha}")
        need(self.focal_gamma > 0, f"Focal gamma must be positive, got {self.focal_gamma}")
        need(self.device in ("cpu", "cuda"), f"Device must be 'cpu' or 'cuda', got {self.device}")
        if self.device == "cuda" and not torch.cuda.is_available():
            print("Warning: CUDA is not available, falling back to CPU")
            self.device = "cpu"

    def update(self, **kwargs):
        for k, v in kwargs.items():
            if not hasattr(self, k):
                raise ValueError(f"Invalid configuration parameter: {k}")
            setattr(self, k, v)
        self.validate()

    def to_dict(self) -> Dict[str, Any]:
        return dict(self.__dict__)

    def save(self, filepath: str):
        os.makedirs(os.path.dirname(os.path.abspath(filepath)), exist_ok=True)
        with open(filepath, "w") as f:
            json.dump(self.to_dict(), f, indent=2)

    @classmethod
    def from_dict(cls, config_dict: Dict[str, Any]) -> "TAGANConfig":
        cfg = cls()
        for k, v in config_dict.items():
            if not hasattr(cfg, k):
                raise ValueError(f"Invalid configuration parameter: {k}")
            setattr(cfg, k, v)
        cfg.validate()
        return cfg

    @classmethod
    def load(cls, filepath: str) -> "TAGANConfig":
        with open(filepath) as f:
            return cls.from_dict(json.load(f))

    def __repr__(self) -> str:
        return "TAGANConfig(\n" + "".join(f"  {k}={v},\n" for k, v in sorted(self.__dict__.items())) + ")"
