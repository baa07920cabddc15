"""Gradient-ready notification for ops that accumulate parameter gradients
themselves (e.g. the fused LoRA backward writes dA/dB straight into the flat
grad buffer with beta=1 GEMMs instead of returning them to autograd).
Such ops call ``mark_ready(p)``; DDP registers ``p._mx_on_grad_ready``."""


def mark_ready(p) -> None:
    h = getattr(p, "_mx_on_grad_ready", None)
    if h is not None:
        h(p)


def direct_grad(p):
    """The preallocated .grad of ``p`` if it can be accumulated into in place
    (never for a parameter used twice in the graph, e.g. a tied embedding/head:
    its gradient is complete only after autograd summed both uses)."""
    if getattr(p, "_mx_no_direct", False):
        return None
    g = p.grad
    if g is not None and g.shape == p.shape and g.dtype == p.dtype and g.is_contiguous():
        return g
    return None


def direct_grad32(p):
    """The fp32 gradient target of ``p`` when its owner accumulates gradients in
    fp32 (``FlatParams(grad_dtype=float32)``, ZeRO-3 fp32 units): ops that form a
    parameter gradient themselves (dW GEMMs with an fp32 output, the RMSNorm dγ and
    embedding kernels' fp32 partials) add into it without an intermediate bf16
    rounding.  None otherwise."""
    if getattr(p, "_mx_no_direct", False):
        return None
    return getattr(p, "_mx_grad32", None)


def accum_grad(p, g) -> bool:
    """Add a computed gradient ``g`` (any float dtype, e.g. the fp32 partials of the
    RMSNorm dγ / embedding kernels) into ``p``'s owner-attached target — the fp32
    one, else the preallocated ``.grad`` — with ONE rounding, and notify the owner.
    A target flagged ``_mx_grad_fresh`` is overwritten (it was not zero-filled).
    False when ``p`` has no such target (return ``g`` to autograd)."""
    if p is None:
        return False
    t = direct_grad32(p)
    if t is None:
        t = direct_grad(p)
    if t is None:
        return False
    if getattr(p, "_mx_grad_fresh", False):
        t.copy_(g.reshape(t.shape))
        p._mx_grad_fresh = False
    else:
        t.add_(g.reshape(t.shape))
    mark_ready(p)
    return True


def deliver_grad(p, g) -> bool:
    """Hand a freshly computed full gradient ``g`` of ``p`` to its owner instead
    of autograd (ZeRO-3 sets ``p._mx_grad_sink`` on parameters whose storage is
    released between uses, where AccumulateGrad would need the full-shape
    parameter).  True when the owner took it (return None to autograd then)."""
    sink = getattr(p, "_mx_grad_sink", None) if p is not None else None
    if sink is None:
        return False
    sink(p, g)
    return True
