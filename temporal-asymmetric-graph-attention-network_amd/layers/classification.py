"""Classification head and loss used by TAGAN (restated from src/tagan/layers/classification.py).

Host-side PyTorch on the GPU (too small for a kernel): attention
pooling over T then Linear -> LN -> ReLU -> Dropout -> Linear
(classification.py:743-975), ``ClassificationModule`` (:1069-1231) and the
loss plumbing ``TemporalLossFunction``/``TemporalLossModule`` (:349-740).
Parameter names match (``classification_head.classification_head.*``).
"""
from typing import Any, Dict, Optional, Union

import torch
import torch.nn as nn
import torch.nn.functional as F


class TemporalLossFunction:
    def __init__(self, task_type: str = "classification", reduction: str = "mean", pos_weight=None,
                 class_weights=None, focal_gamma: float = 2.0, focal_alpha=None, temporal_discount: float = 1.0,
                 huber_delta: float = 1.0, quantile_tau: float = 0.5):
        self.task_type, self.reduction = task_type, reduction
        self.pos_weight, self.class_weights = pos_weight, class_weights
        self.focal_gamma, self.focal_alpha = focal_gamma, focal_alpha
        self.temporal_discount, self.huber_delta, self.quantile_tau = temporal_discount, huber_delta, quantile_tau

    def __call__(self, predictions, targets, time_weights=None, mask=None):
        if self.task_type in ("classification", "focal") and predictions.size(-1) == 1:
            if predictions.dim() == 2 and predictions.size(1) == 1 and targets.dim() == 1 and \
                    predictions.size(0) == targets.size(0):
                predictions = predictions.squeeze(-1)
            elif predictions.size(0) == 1 and targets.dim() == 1:
                predictions = predictions.squeeze(-1).expand(targets.size(0))
            elif predictions.dim() == 1 and targets.dim() == 2 and predictions.size(0) == targets.size(0):
                targets = targets.squeeze(-1)
            elif predictions.size(0) == 1 and targets.dim() == 2:
                predictions = predictions.expand(targets.size(0), -1)
        if self.task_type in ("multi_class", "classification") and predictions.dim() == 2 and \
                predictions.size(1) > 1 and targets.dim() == 1:
            pass
        elif predictions.shape != targets.shape:
            raise ValueError(f"Predictions shape {predictions.shape} does not match targets shape "
                             f"{targets.shape} after attempted reshaping")
        t = self.task_type
        if t == "classification":
            loss = F.binary_cross_entropy_with_logits(predictions, targets, pos_weight=self.pos_weight,
                                                      reduction="none")
        elif t == "multi_class":
            if predictions.size(-1) == targets.size(-1):
                targets = targets.argmax(dim=-1)
            shp = predictions.shape
            loss = F.cross_entropy(predictions.view(-1, shp[-1]), targets.view(-1), weight=self.class_weights,
                                   reduction="none").view(*shp[:-1])
        elif t == "multi_label":
            loss = F.binary_cross_entropy_with_logits(predictions, targets, reduction="none")
        elif t == "focal":
            if predictions.size(-1) == 1:
                probs = torch.sigmoid(predictions)
                p_t = torch.where(targets == 1, probs, 1 - probs)
                alpha_t = (torch.where(targets == 1, self.focal_alpha, 1 - self.focal_alpha)
                           if self.focal_alpha is not None else torch.ones_like(p_t))
                base = F.binary_cross_entropy_with_logits(predictions, targets, reduction="none")
            else:
                probs = F.softmax(predictions, dim=-1)
                oh = F.one_hot(targets, predictions.size(-1)).float() if targets.dim() == predictions.dim() - 1 \
                    else targets
                p_t = torch.sum(probs * oh, dim=-1)
                if self.focal_alpha is None:
                    alpha_t = torch.ones_like(p_t)
                elif not isinstance(self.focal_alpha, torch.Tensor):
                    alpha_t = torch.ones_like(p_t) * self.focal_alpha
                else:
                    alpha_t = torch.sum(self.focal_alpha.unsqueeze(0) * oh, dim=-1)
                base = F.cross_entropy(predictions, targets, weight=self.class_weights, reduction="none")
            loss = alpha_t * (1 - p_t) ** self.focal_gamma * base
        elif t == "huber":
            loss = F.smooth_l1_loss(predictions, targets, beta=self.huber_delta, reduction="none")
        elif t == "quantile":
            diff = targets - predictions
            loss = torch.max(self.quantile_tau * diff, (self.quantile_tau - 1) * diff)
        else:
            loss = F.mse_loss(predictions, targets, reduction="none")
        if mask is not None:
            loss = loss * mask
        if time_weights is not None:
            while time_weights.dim() < loss.dim():
                time_weights = time_weights.unsqueeze(-1)
            loss = loss * time_weights
        if self.reduction == "mean":
            return loss.sum() / (mask.sum() + 1e-8) if mask is not None else loss.mean()
        if self.reduction == "sum":
            return loss.sum()
        return loss


class TemporalLossModule(nn.Module):
    def __init__(self, task_configs: Dict[str, Dict[str, Any]], loss_config: Optional[Dict[str, Any]] = None,
                 default_task_type: str = "classification", default_reduction: str = "mean"):
        super().__init__()
        self.task_configs = task_configs
        self.loss_config = loss_config or {}
        self.default_task_type = default_task_type
        self.default_reduction = self.loss_config.get("reduction", default_reduction)
        self.loss_functions, self.task_weights = {}, {}
        for name, cfg in task_configs.items():
            g = lambda k, d=None: cfg.get(k, self.loss_config.get(k, d))  # noqa: E731
            pw, cw = g("pos_weight"), g("class_weights")
            if pw is not None and not isinstance(pw, torch.Tensor):
                pw = torch.tensor(pw)
            if cw is not None and not isinstance(cw, torch.Tensor):
                cw = torch.tensor(cw)
            self.loss_functions[name] = TemporalLossFunction(
                task_type=cfg.get("task_type", default_task_type),
                reduction=cfg.get("reduction", self.default_reduction), pos_weight=pw, class_weights=cw,
                focal_gamma=g("focal_gamma", 2.0), focal_alpha=g("focal_alpha"),
                temporal_discount=g("temporal_discount", 1.0), huber_delta=g("huber_delta", 1.0),
                quantile_tau=g("quantile_tau", 0.5))
            self.task_weights[name] = cfg.get("loss_weight", 1.0)
        self.default_loss_fn = TemporalLossFunction(task_type=default_task_type, reduction=default_reduction)

    def forward(self, predictions, targets, time_weights=None, masks=None, return_task_losses=False):
        if isinstance(predictions, dict) and isinstance(targets, dict):
            losses = {}
            for name, pred in predictions.items():
                fn = self.loss_functions.get(name)
                if name in targets and fn is not None:
                    losses[name] = self.task_weights.get(name, 1.0) * fn(
                        pred, targets[name], time_weights=time_weights.get(name) if time_weights else None,
                        mask=masks.get(name) if masks else None)
        else:
            losses = {"default": self.default_loss_fn(predictions, targets)}
        total = sum(losses.values())
        return (total, losses) if return_task_losses else total


class TemporalClassificationHead(nn.Module):
    def __init__(self, hidden_dim: int, num_classes: int, pooling_type: str = "attention", dropout: float = 0.1,
                 activation: str = "relu", num_layers: int = 2, use_layer_norm: bool = True,
                 multi_label: bool = False, class_weights: Optional[torch.Tensor] = None):
        super().__init__()
        self.hidden_dim, self.num_classes, self.pooling_type = hidden_dim, num_classes, pooling_type
        self.dropout, self.activation, self.num_layers = dropout, activation, num_layers
        self.use_layer_norm, self.multi_label = use_layer_norm, multi_label
        if pooling_type == "attention":
            self.attention = nn.Sequential(nn.Linear(hidden_dim, hidden_dim), nn.Tanh(),
                                           nn.Linear(hidden_dim, 1, bias=False))
        acts = {"relu": nn.ReLU, "leaky_relu": nn.LeakyReLU, "gelu": nn.GELU, "elu": nn.ELU}
        layers = []
        for i in range(num_layers):
            out_f = num_classes if i == num_layers - 1 else hidden_dim
            layers.append(nn.Linear(hidden_dim, out_f))
            if i < num_layers - 1:
                if use_layer_norm:
                    layers.append(nn.LayerNorm(out_f))
                layers.append(acts.get(activation, nn.ReLU)())
                layers.append(nn.Dropout(dropout))
        self.classifier = nn.Sequential(*layers)
        self.loss_fn = (nn.BCEWithLogitsLoss(reduction="mean", pos_weight=class_weights) if multi_label
                        else nn.CrossEntropyLoss(reduction="mean", weight=class_weights))
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)

    def _pool_temporal(self, x, mask=None):
        pt = self.pooling_type
        if pt == "max":
            if mask is not None:
                me = mask.unsqueeze(-1).float()
                return (x * me + (1 - me) * -1e9).max(dim=1)[0]
            return x.max(dim=1)[0]
        if pt == "last":
            if mask is not None:
                idx = torch.clamp(mask.sum(dim=1, keepdim=True).long() - 1, min=0)
                return x[torch.arange(x.size(0)).unsqueeze(1), idx.view(-1, 1).expand(-1, x.size(-1))].squeeze(1)
            return x[:, -1]
        if pt == "first":
            return x[:, 0]
        if pt == "attention":
            s = self.attention(x)
            if mask is not None:
                me = mask.unsqueeze(-1).float()
                s = s * me + (1 - me) * -1e9
            return (x * F.softmax(s, dim=1)).sum(dim=1)
        if mask is not None:
            me = mask.unsqueeze(-1).float()
            return (x * me).sum(dim=1) / (me.sum(dim=1) + 1e-10)
        return x.mean(dim=1)

    def forward(self, x, mask=None, labels=None):
        logits = self.classifier(self._pool_temporal(x, mask))
        if labels is None:
            return logits
        if self.multi_label and labels.dim() == 1:
            labels = F.one_hot(labels, num_classes=self.num_classes).float()
        return self.loss_fn(logits, labels), logits


class FusedHeadFn(torch.autograd.Function):
    """graph_features (row 0 = x0 [T, H], rows 1..B-1 zero) -> logits, predictions, loss in ONE kernel each way
    (csrc/head.hip, tagan_head_fwd/bwd): attention pooling, Linear -> LN -> ReLU -> Dropout -> Linear, sigmoid or
    softmax, BCE-with-logits / cross-entropy mean (classification.py:856-966, model.py:430-459)."""

    @staticmethod
    def forward(ctx, x0, W1, b1, w2, Wc1, bc1, lnw, lnb, Wc2, bc2, B: int, eps: float, p_drop: float, seed: int,
                labels, loss_kind: int):
        from .._lib import check, lib, ptr, stream_of
        T, H = x0.shape
        C = Wc2.shape[0]
        dev = x0.device
        L = lib()
        logits = torch.empty(B, C, device=dev)
        preds = torch.empty(B, C, device=dev)
        loss = torch.empty(1, device=dev) if loss_kind else None
        saved = torch.empty(int(L.tagan_head_saved_floats(B, T, H)), device=dev)
        # x0, W1, Wc1 go to the kernel as float4 runs (tagan_head_fwd refuses pointers off 16 bytes): a view at an
        # odd offset is copied
        ps = [t.detach().contiguous() for t in (x0, W1, b1, w2, Wc1, bc1, lnw, lnb, Wc2, bc2)]
        ps = [t.clone() if i in (0, 1, 4) and t.data_ptr() % 16 else t for i, t in enumerate(ps)]
        check(L.tagan_head_fwd(B, T, H, C, *[ptr(t) for t in ps[:8]], float(eps), ptr(ps[8]), ptr(ps[9]),
                               float(p_drop), seed, ptr(labels), int(loss_kind), ptr(logits), ptr(preds), ptr(loss),
                               ptr(saved), stream_of(x0)), "tagan_head_fwd")
        ctx.save_for_backward(*ps, logits, preds, saved, labels)
        ctx.cfg = (B, p_drop, seed, loss_kind)
        if loss is None:
            return logits, preds
        return logits, preds, loss.reshape(())

    @staticmethod
    def backward(ctx, g_logits, g_preds, g_loss=None):
        from .._lib import check, lib, ptr, stream_of
        x0, W1, b1, w2, Wc1, bc1, lnw, lnb, Wc2, bc2, logits, preds, saved, labels = ctx.saved_tensors
        B, p_drop, seed, loss_kind = ctx.cfg
        T, H = x0.shape
        C = Wc2.shape[0]
        grads = [torch.empty_like(t) for t in (x0, W1, b1, w2, Wc1, bc1, lnw, lnb, Wc2, bc2)]
        c = lambda g: None if g is None else g.contiguous()  # noqa: E731
        gl = c(g_loss.reshape(1)) if g_loss is not None else None
        check(lib().tagan_head_bwd(B, T, H, C, ptr(x0), ptr(W1), ptr(w2), ptr(Wc1), ptr(lnw), ptr(lnb), ptr(Wc2),
                                   float(p_drop), seed, ptr(labels), int(loss_kind), ptr(logits), ptr(preds),
                                   ptr(saved), ptr(gl), ptr(c(g_logits)), ptr(c(g_preds)),
                                   *[ptr(g) for g in grads], stream_of(x0)), "tagan_head_bwd")
        return (*grads, None, None, None, None, None, None)


def fused_head(module: "ClassificationModule", pooled: torch.Tensor, batch_size: int,
               labels: Optional[torch.Tensor], output_dim: int, seed: Optional[int] = None):
    """(logits, predictions, loss) of TAGAN.head through FusedHeadFn, or None when this head / loss form is not
    the one the kernel implements (attention pooling, 2 layers with LayerNorm + ReLU, BCE or CE) — the caller
    then runs the module path, which also reproduces the reference's errors for unsupported label shapes."""
    from .._lib import lib
    from ..kernels import new_seed
    head = getattr(module, "classification_head", None)
    if not (pooled.is_cuda and pooled.dtype == torch.float32 and isinstance(head, TemporalClassificationHead)
            and head.pooling_type == "attention" and head.num_layers == 2 and head.use_layer_norm
            and head.activation == "relu" and not head.multi_label):
        return None
    T, H = pooled.shape
    C = head.num_classes
    if not lib().tagan_head_supported(T, H, C):
        return None
    lin1, ln, _relu, drop, lin2 = head.classifier
    att1, _tanh, att2 = head.attention
    loss_kind, lab = 0, None
    if labels is not None:
        if labels.dtype == torch.bool:
            labels = labels.long()
        if output_dim > 1 and labels.dim() == 1:                     # model.py:439-441
            if labels.shape[0] != batch_size or labels.is_floating_point():
                return None
            loss_kind, lab = 2, labels.to(torch.float32).contiguous()
        else:                                                        # TemporalLossModule default: BCE mean
            ok = labels.is_floating_point() and (
                (C == 1 and labels.dim() == 1 and labels.shape[0] == batch_size) or
                (labels.dim() == 2 and tuple(labels.shape) == (batch_size, C)))
            if not ok:
                return None
            loss_kind, lab = 1, labels.to(torch.float32).contiguous()
    p = drop.p if head.training else 0.0
    s = (seed if seed is not None else new_seed()) if p > 0 else 0
    out = FusedHeadFn.apply(pooled, att1.weight, att1.bias, att2.weight.reshape(-1), lin1.weight, lin1.bias,
                            ln.weight, ln.bias, lin2.weight, lin2.bias, batch_size, ln.eps, p, s, lab, loss_kind)
    if loss_kind:
        return out
    return out[0], out[1], None


class ClassificationModule(nn.Module):
    """Single-task form used by TAGAN (classification.py:1069-1231; multi-task head not restated)."""

    def __init__(self, hidden_dim: int, task_configs: Union[Dict[str, Any], int], pooling_type: str = "attention",
                 dropout: float = 0.1, activation: str = "relu", num_layers: int = 2, use_layer_norm: bool = True,
                 multi_task: bool = False, class_weights: Optional[torch.Tensor] = None):
        super().__init__()
        self.hidden_dim, self.multi_task = hidden_dim, multi_task
        if isinstance(task_configs, int):
            self.task_configs = {"default": {"output_dim": task_configs, "task_type": "classification"}}
        elif isinstance(task_configs, dict):
            self.task_configs = {"default": task_configs} if "output_dim" in task_configs else task_configs
        else:
            raise ValueError("task_configs must be either int (num_classes) or dict")
        if multi_task:
            raise NotImplementedError("MultiTaskPredictionHead is outside the ported hot path (SURVEY.md §2)")
        cfg = self.task_configs.get("default", next(iter(self.task_configs.values())))
        self.classification_head = TemporalClassificationHead(
            hidden_dim=hidden_dim, num_classes=cfg.get("output_dim", 1), pooling_type=pooling_type,
            dropout=dropout, activation=activation, num_layers=num_layers, use_layer_norm=use_layer_norm,
            multi_label=cfg.get("task_type", "classification") == "multi_label", class_weights=class_weights)

    def forward(self, x, mask=None, labels=None, tasks=None):
        return self.classification_head(x, mask, labels)
