"""Gradient-ready notification for ops that accumulate parameter gradients
themselves (e.g. the fused LoRA backward writes dA/dB straight into the flat
grad buffer with beta=1 GEMMs instead of returning them to autograd).
Such ops call ``mark_ready(p)``; DDP registers ``p._mx_on_grad_ready``."""


def mark_ready(p) -> None:
    h = getattr(p, "_mx_on_grad_ready", None)
    if h is not None:
        h(p)


def direct_grad(p):
    """The preallocated .grad of ``p`` if it can be accumulated into in place."""
    g = p.grad
    if g is not None and g.shape == p.shape and g.dtype == p.dtype and g.is_contiguous():
        return g
    return None
