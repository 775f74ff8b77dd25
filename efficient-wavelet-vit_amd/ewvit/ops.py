"""Torch-facing ops over the C-ABI (include/ewvit.h) and their autograd Functions.

torch is plumbing here: it owns device memory (caching allocator), the current
HIP stream and autograd.  Every FLOP of these ops runs in libewvit.so; inputs
on a non-ROCm device raise (no CPU path).
"""
import math
import os
from typing import Optional, Tuple

import torch

from . import _lib as L
from . import bn as _bn
from . import defer as _defer
from . import grads
from .grads import grad_out, note_use

F32, BF16 = L.F32, L.BF16


def _seed():
    # CPU generator: no device sync, reproducible under torch.manual_seed
    return int(torch.randint(1, 2 ** 62, (), dtype=torch.int64))


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


# ------------------------------------------------------------------- GEMM
def gemm(A, lda, B, ldb, C, M, N, K, *, alpha=1.0, beta=0.0, bias=None, act=0, aux=None,
         drop_p=0.0, seed=0, seed_offset=None, resid=None, ldr=0, splitk=None, fp8=False):
    """Raw C[M,N] = epi(alpha * A(M,K) @ B(K,N)).  lda = (lda_m, lda_k), ldb = (ldb_k, ldb_n).
    C must be contiguous with row stride N (ldc = C.stride(0)).
    fp8=True: MXFP8 operands — every 32-element K run of a row of A / column of B rounded to
    OCP e4m3 under its own power-of-two scale (ewvit_gemm_mx8, include/ewvit.h)."""
    L.require_gpu(A, B, C)
    if splitk is None:
        tiles = ((M + 63) // 64) * ((N + 63) // 64)
        splitk = 1
        # small grids (the ViT / DAMA token GEMMs: M, N <= 512) are latency-bound on
        # their serial K loop: split K so ~256 workgroups run >= 8 K-steps of 32 each
        if tiles < 128 and K >= 256:
            splitk = int(max(1, min(64, 512 // max(tiles, 1), K // 128)))
    ws = torch.empty(splitk * M * N, dtype=torch.float32, device=C.device) if splitk > 1 else None
    work = {'flops': 2.0 * M * N * K,
            'bytes': M * K * A.element_size() + K * N * B.element_size() + M * N * C.element_size()}
    args = (L.ptr(A), L.dt(A), lda[0], lda[1], L.ptr(B), L.dt(B), ldb[0], ldb[1],
            L.ptr(C), L.dt(C), C.stride(0), M, N, K, float(alpha), float(beta), L.ptr(bias), act,
            L.ptr(aux), float(drop_p), seed, L.ptr(seed_offset), L.ptr(resid),
            L.dt(resid) if resid is not None else 0, ldr, splitk, L.ptr(ws))
    L.call('ewvit_gemm_mx8' if fp8 else 'ewvit_gemm', *args, L.stream(C), work=work)
    return C


def _tallk(X, W, out, kw):
    """The few-row, long-K shape class of ewvit_gemm_tallk (patch_to_embedding's forward,
    sfe.py:155): bf16 X with at most 64 rows, fp32 W, K and N multiples of 256, K >= 16384,
    fp32 output, no epilogue but a bias."""
    M, K = X.shape
    N = W.shape[0]
    def unset(v):
        return v is None or (isinstance(v, (bool, int, float)) and not v)
    if not all(unset(v) for k, v in kw.items() if k != 'bias'):
        return False
    return (M <= 64 and K >= 16384 and K % 256 == 0 and N % 256 == 0 and X.dtype == torch.bfloat16
            and W.dtype == torch.float32 and W.is_contiguous() and X.stride(0) % 8 == 0 and out.dtype == torch.float32
            and out.stride(1) == 1)


def mm_nt(X, W, out, **kw):
    """out[M,N] = X[M,K] @ W[N,K]^T  (nn.Linear forward)."""
    M, K = X.shape
    N = W.shape[0]
    assert X.stride(1) == 1 and W.stride(1) == 1
    if not kw.get('fp8') and _tallk(X, W, out, kw):
        L.require_gpu(X, W, out)
        ws = torch.empty(int(L.load().ewvit_gemm_tallk_workspace(M, N, K)) // 4, dtype=torch.float32, device=X.device)
        bias = kw.get('bias')
        L.call('ewvit_gemm_tallk', L.ptr(X), X.stride(0), L.ptr(W), L.ptr(bias), L.ptr(out), out.stride(0), M, N, K,
               L.ptr(ws), L.stream(out), work={'flops': 2.0 * M * N * K, 'bytes': M * K * 2 + N * K * 4 + M * N * 4})
        return out
    return gemm(X, (X.stride(0), 1), W, (1, W.stride(0)), out, M, N, K, **kw)


def mm_nn(G, W, out, **kw):
    """out[M,K] = G[M,N] @ W[N,K]  (input gradient of nn.Linear)."""
    M, N = G.shape
    K = W.shape[1]
    assert G.stride(1) == 1 and W.stride(1) == 1
    return gemm(G, (G.stride(0), 1), W, (W.stride(0), 1), out, M, K, N, **kw)


def mm_tn(G, X, out, **kw):
    """out[N,K] = G[M,N]^T @ X[M,K]  (weight gradient of nn.Linear)."""
    M, N = G.shape
    K = X.shape[1]
    assert G.stride(1) == 1 and X.stride(1) == 1
    return gemm(G, (1, G.stride(0)), X, (X.stride(0), 1), out, N, K, M, **kw)


def colsum(X, out, accumulate=False):
    M, N = X.shape
    L.call('ewvit_colsum', L.ptr(X), L.dt(X), X.stride(0), M, N, L.ptr(out), int(accumulate), L.stream(X))
    return out


# ------------------------------------------------------------- custom ops
# The hot-path ops of the north_star (projection / MLP GEMMs, LayerNorm, attention, the DWT
# front end) are torch.library custom ops in the `ewvit` namespace (torch.ops.ewvit.*): a real
# implementation launching the C-ABI, a fake (meta) implementation so FakeTensor and
# torch.compile trace through them without running kernels, and autograd registered with
# torch.library.register_autograd whose backward is itself made of ewvit custom ops.

_EMPTY = (0,)


def _seed_for(drop_p):
    return _seed() if drop_p > 0 else 0


@torch.library.custom_op('ewvit::linear', mutates_args=())
def _linear_op(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], act: int, drop_p: float,
               seed: int, resid: Optional[torch.Tensor], out_dtype: torch.dtype, fp8: bool,
               need_aux: bool) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """y = dropout(act(x @ W^T + b)) + resid — nn.Linear (+ReLU/GELU/Dropout/residual) of
    network/sfe.py:29-55,127,134-142 and network/dama.py:25-31,105-113.
    -> (y [*, N], aux = bf16 pre-activation [M, N] (act 1/2 with need_aux, else empty),
        an empty float tensor (the per-tensor fp8 amax slot of ABI 2; MXFP8 needs none))."""
    L.require_gpu(x, weight)
    K = x.shape[-1]
    lead = x.shape[:-1]
    x2 = _c(x.reshape(-1, K))
    M, N = x2.shape[0], weight.shape[0]
    y = torch.empty(M, N, dtype=out_dtype, device=x.device)
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=x.device) if (need_aux and act in (1, 2)) else None
    soff = L.rng_offset(x.device) if drop_p > 0 else None
    r2 = _c(resid.reshape(M, N)) if resid is not None else None
    mm_nt(x2, _c(weight), y, bias=bias, act=act, aux=aux, drop_p=drop_p, seed=seed, seed_offset=soff,
          resid=r2, ldr=N if r2 is not None else 0, fp8=fp8)
    e = x.new_empty(_EMPTY, dtype=torch.float32)
    return y.reshape(*lead, N), (aux if aux is not None else e.to(torch.bfloat16)), e.clone()


@_linear_op.register_fake
def _(x, weight, bias, act, drop_p, seed, resid, out_dtype, fp8, need_aux):
    M = x.numel() // x.shape[-1]
    N = weight.shape[0]
    aux = x.new_empty((M, N) if (need_aux and act in (1, 2)) else _EMPTY, dtype=torch.bfloat16)
    xa = x.new_empty(_EMPTY, dtype=torch.float32)
    return x.new_empty((*x.shape[:-1], N), dtype=out_dtype), aux, xa


@torch.library.custom_op('ewvit::linear_backward', mutates_args=('dw_out', 'db_out'))
def _linear_backward_op(dy: torch.Tensor, x: torch.Tensor, weight: torch.Tensor, aux: torch.Tensor,
                        xa: torch.Tensor, act: int, drop_p: float, seed: int, need_dx: bool, fp8: bool,
                        dw_out: Optional[torch.Tensor], db_out: Optional[torch.Tensor]) -> torch.Tensor:
    """dX (x's dtype; empty unless need_dx), dW into dw_out and db into db_out when given
    (gradient slots of the data-parallel flat buffer, ewvit.grads)."""
    K = x.shape[-1]
    x2 = _c(x.reshape(-1, K))
    M, N = x2.shape[0], weight.shape[0]
    dy2 = _c(dy.reshape(M, N))
    if act == 0 and drop_p == 0:
        g = dy2
    else:
        g = torch.empty(M, N, dtype=torch.float32, device=dy.device)
        soff = L.rng_offset(dy.device) if drop_p > 0 else None
        L.call('ewvit_act_bwd', L.ptr(dy2), L.dt(dy2), N, L.ptr(aux) if aux.numel() else None, act,
               float(drop_p), seed, L.ptr(soff), L.ptr(g), F32, M, N, L.stream(g))
    dx = dy.new_empty(_EMPTY, dtype=x.dtype)
    if need_dx:
        dx = mm_nn(g, _c(weight), torch.empty(M, K, dtype=x.dtype, device=dy.device), fp8=fp8).reshape(x.shape)
    if dw_out is not None:
        dw = dw_out if dw_out.is_contiguous() else torch.empty(N, K, dtype=torch.float32, device=dy.device)
        mm_tn(g, x2, dw, fp8=fp8)
        if dw is not dw_out:
            dw_out.copy_(dw)
    if db_out is not None:
        colsum(g, db_out)
    return dx


@_linear_backward_op.register_fake
def _(dy, x, weight, aux, xa, act, drop_p, seed, need_dx, fp8, dw_out, db_out):
    return dy.new_empty(x.shape if need_dx else _EMPTY, dtype=x.dtype)


def _linear_setup(ctx, inputs, output):
    x, weight, bias, act, drop_p, seed, resid, out_dtype, fp8, need_aux = inputs
    _, aux, xa = output
    ctx.mark_non_differentiable(aux, xa)
    ctx.set_materialize_grads(False)     # no zero-filled gradients for aux / xa
    ctx.save_for_backward(x, weight, aux, xa)
    ctx.params = (weight, bias)          # gradient slots (ewvit.grads) are looked up on these
    ctx.gen = note_use(weight)
    note_use(bias)
    ctx.cfg = (act, drop_p, seed, resid is not None, bias is not None, fp8)


def _linear_backward(ctx, dy, _daux, _dxa):
    if dy is None:
        return (None,) * 10
    x, weight, aux, xa = ctx.saved_tensors
    act, drop_p, seed, has_res, has_bias, fp8 = ctx.cfg
    need = ctx.needs_input_grad
    dw = db = None
    if need[1]:
        dw = grad_out(ctx.params[0], ctx.gen)
    if has_bias and need[2]:
        db = grad_out(ctx.params[1], ctx.gen)
        if db.dim() != 1 or not db.is_contiguous():
            db = torch.empty(db.shape[0], dtype=torch.float32, device=dy.device)
    dx = torch.ops.ewvit.linear_backward(dy, x, weight, aux, xa, act, drop_p, seed, bool(need[0]), fp8, dw, db)
    dres = dy if has_res and need[6] else None
    dw = grads.give(ctx.params[0], dw, ctx.gen)
    db = grads.give(ctx.params[1], db, ctx.gen)
    return (dx if need[0] else None), dw, db, None, None, None, dres, None, None, None


_linear_op.register_autograd(_linear_backward, setup_context=_linear_setup)


def linear(x, weight, bias=None, act=0, drop_p=0.0, resid=None, out_dtype=torch.float32, fp8=False):
    """torch.ops.ewvit.linear with autograd.  act 0 none / 1 GELU(erf) / 2 ReLU; dropout and
    the residual add fused in the GEMM epilogue.  fp8=True: the forward and both backward
    GEMMs take MXFP8 operands (OCP e4m3, one power-of-two scale per 32 K elements; BASELINE
    configs[4]); the epilogue (bias, activation, dropout, residual) is fp32."""
    drop_p = float(drop_p)
    need_aux = act in (1, 2) and torch.is_grad_enabled() and (
        x.requires_grad or weight.requires_grad or (bias is not None and bias.requires_grad))
    y, _, _ = torch.ops.ewvit.linear(x, weight, bias, int(act), drop_p, _seed_for(drop_p), resid, out_dtype,
                                     bool(fp8), bool(need_aux))
    return y


# -------------------------------------------------------------- LayerNorm
@torch.library.custom_op('ewvit::layer_norm', mutates_args=())
def _layer_norm_op(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float,
                   out_dtype: torch.dtype) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """nn.LayerNorm over the last dim (network/sfe.py:23, network/dama.py:62,64) -> (y, mean, rstd)."""
    L.require_gpu(x, weight)
    D = x.shape[-1]
    x2 = _c(x.reshape(-1, D))
    M = x2.shape[0]
    y = torch.empty(M, D, dtype=out_dtype, device=x.device)
    mean = torch.empty(M, dtype=torch.float32, device=x.device)
    rstd = torch.empty_like(mean)
    L.call('ewvit_layernorm_fwd', L.ptr(x2), L.dt(x2), D, L.ptr(weight), L.ptr(bias), L.ptr(y),
           L.dt(y), L.ptr(mean), L.ptr(rstd), M, D, float(eps), L.stream(y))
    return y.reshape(x.shape), mean, rstd


@_layer_norm_op.register_fake
def _(x, weight, bias, eps, out_dtype):
    M = x.numel() // x.shape[-1]
    return (x.new_empty(x.shape, dtype=out_dtype), x.new_empty((M,), dtype=torch.float32),
            x.new_empty((M,), dtype=torch.float32))


@torch.library.custom_op('ewvit::layer_norm_backward', mutates_args=())
def _layer_norm_backward_op(dy: torch.Tensor, x: torch.Tensor, weight: torch.Tensor, mean: torch.Tensor,
                            rstd: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    D = x.shape[-1]
    x2 = _c(x.reshape(-1, D))
    M = x2.shape[0]
    dy2 = _c(dy.reshape(M, D))
    dx = torch.empty(M, D, dtype=torch.float32, device=dy.device)
    dg = torch.empty(D, dtype=torch.float32, device=dy.device)
    db = torch.empty(D, dtype=torch.float32, device=dy.device)
    ws = torch.empty(L.load().ewvit_layernorm_bwd_workspace(M, D) // 4, dtype=torch.float32, device=dy.device)
    L.call('ewvit_layernorm_bwd', L.ptr(dy2), L.dt(dy2), L.ptr(x2), L.dt(x2), D, L.ptr(weight),
           L.ptr(mean), L.ptr(rstd), L.ptr(dx), 0, L.ptr(dg), L.ptr(db), L.ptr(ws), M, D, L.stream(dx))
    dx = dx.reshape(x.shape)
    return (dx if x.dtype == torch.float32 else dx.to(x.dtype)), dg, db


@_layer_norm_backward_op.register_fake
def _(dy, x, weight, mean, rstd):
    D = x.shape[-1]
    return (x.new_empty(x.shape), x.new_empty((D,), dtype=torch.float32), x.new_empty((D,), dtype=torch.float32))


def _ln_setup(ctx, inputs, output):
    x, weight, _, _, _ = inputs
    _, mean, rstd = output
    ctx.mark_non_differentiable(mean, rstd)
    ctx.set_materialize_grads(False)
    ctx.save_for_backward(x, weight, mean, rstd)
    ctx.gen = note_use(inputs[1])
    note_use(inputs[2])
    ctx.params = (inputs[1], inputs[2])


def _ln_backward(ctx, dy, _dm, _dr):
    if dy is None:
        return (None,) * 5
    x, weight, mean, rstd = ctx.saved_tensors
    dx, dg, db = torch.ops.ewvit.layer_norm_backward(dy, x, weight, mean, rstd)
    return dx, grads.give(ctx.params[0], dg, ctx.gen), grads.give(ctx.params[1], db, ctx.gen), None, None


_layer_norm_op.register_autograd(_ln_backward, setup_context=_ln_setup)


def layer_norm(x, weight, bias, eps=1e-5, out_dtype=torch.bfloat16):
    return torch.ops.ewvit.layer_norm(x, weight, bias, float(eps), out_dtype)[0]


# -------------------------------------------------------------- attention
@torch.library.custom_op('ewvit::attention', mutates_args=())
def _attention_op(q_src: torch.Tensor, kv_src: Optional[torch.Tensor], heads: int, dim_head: int,
                  scale: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """Multi-head softmax attention for the hot path's short sequences -> (o, softmax p).

    packed (ViT, sfe.py:59-70): q_src = qkv [B, n, 3*H*d], kv_src None -> o [B, n, H*d]
    cross (dama.py:41-53):      q_src = q [B, nq, H*d], kv_src = kv [B, nk, 2*H*d]
    """
    packed = kv_src is None
    qs = _c(q_src)
    kvs = qs if packed else _c(kv_src)
    L.require_gpu(qs, kvs)
    if qs.dtype != torch.bfloat16 or kvs.dtype != torch.bfloat16:
        raise TypeError('attn: q/k/v must be bf16 (projection outputs)')
    B, nq = qs.shape[0], qs.shape[1]
    nk = kvs.shape[1]
    inner = heads * dim_head
    o = torch.empty(B, nq, inner, dtype=torch.bfloat16, device=qs.device)
    p = torch.empty(B, heads, nq, nk, dtype=torch.float32, device=qs.device)
    esz = 2
    q_off, k_off, v_off = (0, inner, 2 * inner) if packed else (0, 0, inner)
    L.call('ewvit_attn_fwd', qs.data_ptr() + q_off * esz, qs.stride(0), qs.stride(1), kvs.data_ptr() + k_off * esz,
           kvs.stride(0), kvs.stride(1), kvs.data_ptr() + v_off * esz, kvs.stride(0), kvs.stride(1), L.ptr(o),
           o.stride(0), o.stride(1), L.ptr(p), B, heads, nq, nk, dim_head, float(scale), L.stream(o))
    return o, p


@_attention_op.register_fake
def _(q_src, kv_src, heads, dim_head, scale):
    B, nq = q_src.shape[0], q_src.shape[1]
    nk = nq if kv_src is None else kv_src.shape[1]
    return (q_src.new_empty((B, nq, heads * dim_head), dtype=torch.bfloat16),
            q_src.new_empty((B, heads, nq, nk), dtype=torch.float32))


@torch.library.custom_op('ewvit::attention_backward', mutates_args=())
def _attention_backward_op(do: torch.Tensor, q_src: torch.Tensor, kv_src: Optional[torch.Tensor],
                           p: torch.Tensor, heads: int, dim_head: int,
                           scale: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """-> (d q_src, d kv_src) — the packed form returns its whole qkv gradient first and an
    empty second tensor."""
    packed = kv_src is None
    qs = _c(q_src)
    kvs = qs if packed else _c(kv_src)
    do = _c(do)
    if do.dtype != torch.bfloat16:
        do = do.to(torch.bfloat16)
    inner = heads * dim_head
    q_off, k_off, v_off = (0, inner, 2 * inner) if packed else (0, 0, inner)
    B, nq, nk = qs.shape[0], qs.shape[1], kvs.shape[1]
    dqs = torch.empty_like(qs)
    dkvs = dqs if packed else torch.empty_like(kvs)
    esz = 2
    L.call('ewvit_attn_bwd', L.ptr(do), do.stride(0), do.stride(1),
           qs.data_ptr() + q_off * esz, qs.stride(0), qs.stride(1),
           kvs.data_ptr() + k_off * esz, kvs.stride(0), kvs.stride(1),
           kvs.data_ptr() + v_off * esz, kvs.stride(0), kvs.stride(1), L.ptr(p),
           dqs.data_ptr() + q_off * esz, dkvs.data_ptr() + k_off * esz, dkvs.data_ptr() + v_off * esz,
           B, heads, nq, nk, dim_head, float(scale), L.stream(dqs))
    return dqs, (qs.new_empty(_EMPTY) if packed else dkvs)


@_attention_backward_op.register_fake
def _(do, q_src, kv_src, p, heads, dim_head, scale):
    return (torch.empty_like(q_src), q_src.new_empty(_EMPTY) if kv_src is None else torch.empty_like(kv_src))


def _attn_setup(ctx, inputs, output):
    q_src, kv_src, heads, dim_head, scale = inputs
    _, p = output
    ctx.mark_non_differentiable(p)
    ctx.set_materialize_grads(False)
    ctx.save_for_backward(q_src, kv_src, p)
    ctx.cfg = (heads, dim_head, scale)


def _attn_backward(ctx, do, _dp):
    if do is None:
        return (None,) * 5
    q_src, kv_src, p = ctx.saved_tensors
    dq, dkv = torch.ops.ewvit.attention_backward(do, q_src, kv_src, p, *ctx.cfg)
    return dq, (dkv if kv_src is not None else None), None, None, None


_attention_op.register_autograd(_attn_backward, setup_context=_attn_setup)


def attention_packed(qkv, heads, dim_head, scale):
    return torch.ops.ewvit.attention(qkv, None, int(heads), int(dim_head), float(scale))[0]


def attention_cross(q, kv, heads, dim_head, scale):
    return torch.ops.ewvit.attention(q, kv, int(heads), int(dim_head), float(scale))[0]


# -------------------------------------------------------------------- DWT
def _level_sizes(H, W, levels):
    out = []
    h, w = H, W
    for _ in range(levels):
        h, w = (h + 1) // 2, (w + 1) // 2
        out.append((h, w))
    return out


def _no_grad_input(x):
    if x.requires_grad and torch.is_grad_enabled():
        raise NotImplementedError('ewvit.dwt_haar: no backward (frames never require grad on the '
                                  'training path, SURVEY §8a note 7)')


def _dwt_flat(x, levels, out_dtype):
    """Raw launch: (ll, all levels' bands flat, level sizes)."""
    L.require_gpu(x)
    x = _c(x)
    N, C, H, W = x.shape
    sizes = _level_sizes(H, W, levels)
    total = sum(N * C * 3 * h * w for h, w in sizes)
    yh = torch.empty(total, dtype=out_dtype, device=x.device)
    hL, wL = sizes[-1]
    ll = torch.empty(N, C, hL, wL, dtype=out_dtype, device=x.device)
    work = {'bytes': x.numel() * x.element_size() + (yh.numel() + ll.numel()) * ll.element_size()}
    L.call('ewvit_dwt_haar_fwd', L.ptr(x), L.ptr(yh), L.ptr(ll), N, C, H, W, levels, L.dt(x),
           L.dt(ll), L.stream(ll), work=work)
    return ll, yh, sizes


@torch.library.custom_op('ewvit::dwt_haar', mutates_args=())
def _dwt_haar_op(x: torch.Tensor, levels: int, out_dtype: torch.dtype) -> Tuple[torch.Tensor, torch.Tensor]:
    """-> (ll [N, C, h_L, w_L], every level's bands flat: level l as [N, C, 3, h_l, w_l])."""
    ll, yh, _ = _dwt_flat(x, levels, out_dtype)
    return ll, yh


@_dwt_haar_op.register_fake
def _(x, levels, out_dtype):
    N, C, H, W = x.shape
    sizes = _level_sizes(H, W, levels)
    return (x.new_empty((N, C) + sizes[-1], dtype=out_dtype),
            x.new_empty((sum(N * C * 3 * h * w for h, w in sizes),), dtype=out_dtype))


@torch.library.custom_op('ewvit::hf_upsample', mutates_args=())
def _hf_upsample_op(yh: torch.Tensor, n: int, c: int, h: int, w: int, levels: int, oh: int, ow: int,
                    out_dtype: torch.dtype, out_channels: int) -> torch.Tensor:
    oc = out_channels or 3 * c
    out = torch.empty(levels, n, oh, ow, oc, dtype=out_dtype, device=yh.device)
    nb = sum(n * 3 * c * hh * ww for hh, ww in _level_sizes(h, w, levels))
    work = {'bytes': nb * yh.element_size() + out.numel() * out.element_size()}
    L.call('ewvit_hf_upsample', L.ptr(yh), L.ptr(out), n, c, h, w, levels, oh, ow, L.dt(yh),
           L.dt(out), oc, L.stream(out), work=work)
    return out


@_hf_upsample_op.register_fake
def _(yh, n, c, h, w, levels, oh, ow, out_dtype, out_channels):
    return yh.new_empty((levels, n, oh, ow, out_channels or 3 * c), dtype=out_dtype)


def dwt_haar(x, levels=1, out_dtype=torch.float32):
    """Multi-level Haar DWT (pytorch_wavelets DWTForward J=1 'haar' 'zero' applied
    `levels` times, network/mwt.py:20,76,107-111).  x [N,C,H,W] f32/bf16.
    Returns (ll [N,C,h_L,w_L], [yh_1 .. yh_L]) with yh_l [N,C,3,h_l,w_l]."""
    _no_grad_input(x)
    ll, yh = torch.ops.ewvit.dwt_haar(x, int(levels), out_dtype)
    N, C = x.shape[:2]
    sizes = _level_sizes(x.shape[2], x.shape[3], levels)
    outs, off = [], 0
    for h, w in sizes:
        n = N * C * 3 * h * w
        outs.append(yh[off:off + n].view(N, C, 3, h, w))
        off += n
    return ll, outs


def hf_upsample(yh_flat_levels, N, C, H, W, levels, out_hw, out_dtype=torch.bfloat16, out_channels=0):
    """Bilinear upsample of every level's bands (mwt.py:77-81) -> [L, N, OH, OW, Cout]
    with Cout = out_channels (>= 3C; channels past 3C are zero) or 3C."""
    return torch.ops.ewvit.hf_upsample(yh_flat_levels, int(N), int(C), int(H), int(W), int(levels),
                                       int(out_hw[0]), int(out_hw[1]), out_dtype, int(out_channels))


def dwt_hf_upsample(x, levels, out_hw, out_dtype=torch.bfloat16, band_dtype=torch.bfloat16, out_channels=0):
    """The MWT high-frequency front end for all levels at once: DWT (one read of x)
    then the upsampled, channel-interleaved HF input of hf_conv for every level,
    channels-last: [L, N, OH, OW, 3C] (channel c*3+band; zero-padded to out_channels)."""
    _no_grad_input(x)
    ll, yh = torch.ops.ewvit.dwt_haar(x, int(levels), band_dtype)
    N, C, H, W = x.shape
    return hf_upsample(yh, N, C, H, W, levels, out_hw, out_dtype, out_channels), ll


@torch.library.custom_op('ewvit::dwt_hf_fused', mutates_args=())
def _dwt_hf_fused_op(x: torch.Tensor, levels: int, out_dtype: torch.dtype, out_channels: int) -> torch.Tensor:
    L.require_gpu(x)
    x = _c(x)
    N, C, H, W = x.shape
    out = torch.empty(levels, N, H // 2, W // 2, out_channels, dtype=out_dtype, device=x.device)
    work = {'bytes': x.numel() * x.element_size() + out.numel() * out.element_size()}
    L.call('ewvit_dwt_hf_upsample_fused', L.ptr(x), L.ptr(out), N, C, H, W, levels, L.dt(x), L.dt(out),
           out_channels, L.stream(out), work=work)
    return out


@_dwt_hf_fused_op.register_fake
def _(x, levels, out_dtype, out_channels):
    N, C, H, W = x.shape
    return x.new_empty((levels, N, H // 2, W // 2, out_channels), dtype=out_dtype)


_DWT_FUSED = os.environ.get('EWVIT_DWT_FUSED', '1') != '0'


def dwt_hf_features(x, levels, out_hw, out_dtype=torch.bfloat16, out_channels=0):
    """The MWT's hf_conv input of every level, [L, N, OH, OW, out_channels or 3C] channels-last
    (bands rounded to out_dtype, as dwt_hf_upsample with band_dtype = out_dtype).  ONE launch
    (ewvit_dwt_hf_upsample_fused: the bands stay on chip) when the shape allows it (3 colour
    planes, levels <= 3, H and W multiples of 2^levels, out_hw = (H/2, W/2), W <= 224,
    9-16 channels), otherwise the DWT + upsample launches."""
    _no_grad_input(x)
    N, C, H, W = x.shape
    oc = int(out_channels) or 3 * C
    if _DWT_FUSED and L.load().ewvit_dwt_hf_fused_ok(N, C, H, W, int(levels), int(out_hw[0]), int(out_hw[1]), oc):
        return torch.ops.ewvit.dwt_hf_fused(x, int(levels), out_dtype, oc)
    return dwt_hf_upsample(x, levels, out_hw, out_dtype, out_dtype, out_channels)[0]


# ------------------------------------------------------- depthwise 3x3 conv
# the stride-1 input gradient sums the backward statistics of the BatchNorm before the conv
# (ewvit_dwconv3x3_bwd_data_bn; 0: that BN runs its own reduction pass, A/B)
_DW_BWD_LINK = os.environ.get('EWVIT_DW_BWD_LINK', '1') != '0'
# the linked stride-1 input gradient and the weight gradient in one pass
# (ewvit_dwconv3x3_bwd_fused; 0: two kernels, A/B)
_DW_BWD_FUSED = os.environ.get('EWVIT_DW_BWD_FUSED', '1') != '0'


class DepthwiseConv3x3Fn(torch.autograd.Function):
    """groups=C 3x3 conv, no bias, channels-last (EfficientNetV2-S MBConv depthwise)."""

    @staticmethod
    def forward(ctx, x, weight, stride, pad, bn_stats=None, selink=None):
        L.require_gpu(x, weight)
        # the BN + SE after this conv may hand its dx pass to this backward (ewvit.se.SeDxLink)
        ctx.selink = selink
        N, C, H, W = x.shape
        xc = x.contiguous(memory_format=torch.channels_last)
        w = weight.detach().float().contiguous()
        Ho, Wo = (H + 2 * pad - 3) // stride + 1, (W + 2 * pad - 3) // stride + 1
        y = torch.empty((N, C, Ho, Wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        work = {'bytes': (xc.numel() + y.numel()) * x.element_size(), 'flops': 18.0 * y.numel()}
        if bn_stats is not None:
            # the BatchNorm statistics of y summed on the way (ewvit_bn_fwd_partials)
            shift, part, shift_out = bn_stats
            L.call('ewvit_dwconv3x3_fwd_bn', L.ptr(xc), L.ptr(w), L.ptr(y), N, H, W, C, stride, L.ptr(shift),
                   L.ptr(part), L.ptr(shift_out), L.stream(y), work=work)
        else:
            L.call('ewvit_dwconv3x3_fwd', L.ptr(xc), L.ptr(w), L.ptr(y), N, H, W, C, stride, pad, L.dt(xc),
                   L.stream(y), work=work)
        ctx.save_for_backward(xc, w)
        ctx.cfg = (stride, pad, weight.dtype)
        ctx.wstride = weight.stride()
        ctx.gen = note_use(weight)
        ctx.params = (weight,)
        # the backward statistics of the BatchNorm that produced x, summed by the input gradient:
        # ewvit_dwconv3x3_bwd_data_bn leaves whole-map sums with no row scale, so only the link
        # of a one-group BatchNorm without a drop-path scale
        ctx.bnlink = _bn.take_bwd_link(x, grouped=False, scaled=False) if (
            _DW_BWD_LINK and stride == 1 and pad == 1 and ctx.needs_input_grad[0]) else None
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, w = ctx.saved_tensors
        stride, pad, wdt = ctx.cfg
        N, C, H, W = xc.shape
        bl = ctx.bnlink
        ctx.bnlink = None
        # the BN + SE backward's dx pass left to this conv (ewvit.se.SeDxLink): folded into the
        # fused backward below when it runs, else formed now (dy is its output, not yet written)
        sl, fold = ctx.selink, None
        ctx.selink = None
        if sl is not None and sl.pending(dy):
            rows = int(L.load().ewvit_dwconv3x3_bn_rows(N, H, W, C, stride, 1)) \
                if bl is not None and xc.dtype == torch.bfloat16 and bl.x.shape == xc.shape else 0
            if (ctx.needs_input_grad[0] and ctx.needs_input_grad[1] and 0 < rows <= _bn.BWD_LINK_MAX_ROWS
                    and wdt == torch.float32 and _DW_BWD_FUSED and C % 8 == 0 and stride == 1 and pad == 1
                    and L.has('ewvit_dwconv3x3_bwd_fused_se')):
                fold = sl.take()
            else:
                sl.materialize()
        dyc = dy.contiguous(memory_format=torch.channels_last)
        if dyc.dtype != xc.dtype:
            dyc = dyc.to(xc.dtype)
        dx = dw = None
        if ctx.needs_input_grad[1]:
            # the gradient slot itself when its layout is the kernel's [C][9] (ewvit.grads)
            out = grad_out(ctx.params[0], ctx.gen) if wdt == torch.float32 else None
            direct = out is not None and tuple(out.shape) == (C, 1, 3, 3) and all(
                a == b for a, b, n in zip(out.stride(), (9, 9, 3, 1), out.shape) if n != 1)
            dw = out if direct else torch.empty(C, 1, 3, 3, dtype=torch.float32, device=xc.device)
        wdone = False
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(xc, memory_format=torch.channels_last)
            rows = int(L.load().ewvit_dwconv3x3_bn_rows(N, H, W, C, stride, 1)) \
                if bl is not None and xc.dtype == torch.bfloat16 and bl.x.shape == xc.shape else 0
            if 0 < rows <= _bn.BWD_LINK_MAX_ROWS:
                # dx and the producing BatchNorm(+SiLU)'s backward sums in one pass
                part = torch.empty(rows, 2 * C, dtype=torch.float32, device=xc.device)
                if dw is not None and _DW_BWD_FUSED and C % 8 == 0 and L.has('ewvit_dwconv3x3_bwd_fused'):
                    # ... and the weight gradient, reading dy once
                    wsb = L.load().ewvit_dwconv3x3_bwd_fused_workspace(N, H, W, C)
                    ws = torch.empty(wsb // 4, dtype=torch.float32, device=xc.device)
                    if direct and grads.deferrable(ctx.params[0], dw, ctx.gen) and _defer.available():
                        # dW is read by nobody before the end of the backward (grads.deferrable):
                        # its slab sum rides in a later weight-gradient launch (ewvit.defer)
                        _defer.mark(ws, dw, xc.device)
                    if fold is not None:
                        # ... with the BN + SE backward of this conv's output folded in: dy is the SE
                        # output gradient, the conv's output gradient is formed per window element
                        f = fold
                        L.call('ewvit_dwconv3x3_bwd_fused_se', L.ptr(f.dy), L.ptr(w), L.ptr(dx), L.ptr(xc),
                               L.ptr(dw), 0, N, H, W, C, L.ptr(bl.x), L.ptr(bl.mean), L.ptr(bl.invstd),
                               L.ptr(bl.gamma), L.ptr(bl.beta), bl.act, L.ptr(part), L.ptr(ws), L.ptr(f.z),
                               L.ptr(f.mean), L.ptr(f.invstd), L.ptr(f.gamma), L.ptr(f.beta), f.act, L.ptr(f.row),
                               L.ptr(f.s), L.ptr(f.g), L.stream(dx),
                               work={'bytes': (2 * f.dy.numel() + 3 * dx.numel()) * dx.element_size()})
                    else:
                        L.call('ewvit_dwconv3x3_bwd_fused', L.ptr(dyc), L.ptr(w), L.ptr(dx), L.ptr(xc), L.ptr(dw), 0,
                               N, H, W, C, L.ptr(bl.x), L.ptr(bl.mean), L.ptr(bl.invstd), L.ptr(bl.gamma),
                               L.ptr(bl.beta), bl.act, L.ptr(part), L.ptr(ws), L.stream(dx),
                               work={'bytes': (dyc.numel() + 3 * dx.numel()) * dx.element_size()})
                    wdone = True
                else:
                    L.call('ewvit_dwconv3x3_bwd_data_bn', L.ptr(dyc), L.ptr(w), L.ptr(dx), N, H, W, C, L.ptr(bl.x),
                           L.ptr(bl.mean), L.ptr(bl.invstd), L.ptr(bl.gamma), L.ptr(bl.beta), bl.act, L.ptr(part),
                           L.stream(dx), work={'bytes': (dyc.numel() + 2 * dx.numel()) * dx.element_size()})
                bl.fulfil(part, rows, dx)
            else:
                L.call('ewvit_dwconv3x3_bwd_data', L.ptr(dyc), L.ptr(w), L.ptr(dx), N, H, W, C, stride, pad,
                       L.dt(xc), L.stream(dx), work={'bytes': (dyc.numel() + dx.numel()) * dx.element_size()})
        if dw is not None:
            if not wdone:
                wsb = L.load().ewvit_dwconv3x3_bwd_weight_workspace(N, H, W, C, stride, pad)
                ws = torch.empty(wsb // 4, dtype=torch.float32, device=xc.device)
                L.call('ewvit_dwconv3x3_bwd_weight', L.ptr(xc), L.ptr(dyc), L.ptr(dw), 0, N, H, W, C, stride, pad,
                       L.dt(xc), L.ptr(ws), L.stream(dw),
                       work={'bytes': (dyc.numel() + xc.numel()) * xc.element_size()})
            if wdt != torch.float32:
                dw = dw.to(wdt)
            if not direct and dw.stride() != ctx.wstride:    # keep the parameter's layout (DDP bucket views)
                if all(a == b for a, b, n in zip(dw.stride(), ctx.wstride, dw.shape) if n != 1):
                    dw = dw.as_strided(dw.shape, ctx.wstride)      # same memory, size-1 dims differ only
                else:
                    dw = torch.empty_strided(dw.shape, ctx.wstride, dtype=dw.dtype, device=dw.device).copy_(dw)
            dw = grads.give(ctx.params[0], dw, ctx.gen)
        if fold is not None and not wdone:
            raise RuntimeError('dwconv3x3 backward: the folded BN + SE dx pass did not run')
        return dx, dw, None, None, None, None


def dwconv3x3(x, weight, stride=1, pad=1):
    if torch.is_autocast_enabled('cuda') and x.dtype == torch.float32:
        x = x.to(torch.get_autocast_dtype('cuda'))
    return DepthwiseConv3x3Fn.apply(x, weight, int(stride), int(pad))


def dwconv3x3_bn_stats(x, weight, stride, shift, selink=None):
    """dwconv3x3 (pad 1, bf16) whose kernel also leaves the BatchNorm partial statistics of
    its output centred on `shift` (the BN running mean): (y, part, shifts, nrc) for
    ewvit.bn.batch_norm_act / bn_act_se(..., partials=(part, shifts, nrc)), or None when the
    shape does not take it."""
    if torch.is_autocast_enabled('cuda') and x.dtype == torch.float32:
        x = x.to(torch.get_autocast_dtype('cuda'))
    if x.dtype != torch.bfloat16 or x.dim() != 4 or not x.is_cuda:
        return None
    N, C, H, W = x.shape
    nrc = int(L.load().ewvit_dwconv3x3_bn_rows(N, H, W, C, int(stride), 0))
    if not 0 < nrc <= 256:
        return None
    part = torch.empty(nrc, 2 * C, dtype=torch.float32, device=x.device)
    shifts = torch.empty(C, dtype=torch.float32, device=x.device)
    sh = shift.detach().float().contiguous() if shift is not None else None
    y = DepthwiseConv3x3Fn.apply(x, weight, int(stride), 1, (sh, part, shifts), selink)
    return y, part, shifts, nrc


# ------------------------------------------------------------------- pooling
class MaxPool2Fn(torch.autograd.Function):
    """MaxPool2d(kernel 2, stride 2) on a channels-last tensor (csrc/pool.hip)."""
    @staticmethod
    def forward(ctx, x):
        L.require_gpu(x)
        xc = x.contiguous(memory_format=torch.channels_last)
        N, C, H, W = xc.shape
        y = torch.empty((N, C, H // 2, W // 2), dtype=xc.dtype, device=x.device, memory_format=torch.channels_last)
        arg = torch.empty((N, H // 2, W // 2, C), dtype=torch.uint8, device=x.device)
        L.call('ewvit_maxpool2_fwd', L.ptr(xc), L.ptr(y), L.ptr(arg), L.dt(xc), N, H, W, C, L.stream(y),
               work={'bytes': (xc.numel() + y.numel()) * xc.element_size() + arg.numel()})
        ctx.save_for_backward(arg)
        ctx.shape = (N, C, H, W, xc.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        arg, = ctx.saved_tensors
        N, C, H, W, dt = ctx.shape
        dyc = dy.to(dt).contiguous(memory_format=torch.channels_last)
        dx = torch.empty((N, C, H, W), dtype=dt, device=dy.device, memory_format=torch.channels_last)
        L.call('ewvit_maxpool2_bwd', L.ptr(dyc), L.ptr(arg), L.ptr(dx), L.dt(dyc), N, H, W, C, L.stream(dx),
               work={'bytes': (dx.numel() + dyc.numel()) * dyc.element_size() + arg.numel()})
        return dx


def maxpool2(x):
    """nn.MaxPool2d(2) (stride 2, floor mode) for [N, C, H, W] with C % 8 == 0, f32/bf16."""
    return MaxPool2Fn.apply(x)
