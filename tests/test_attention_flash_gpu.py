"""Flash-style attention (mmdx_attention_fwd_lse / mmdx_attention_bwd_lse) vs torch fp32 and
vs the P-saving kernels it replaces on the benched path.

The forward is the P-saving kernel with the row log-sum-exp written instead of P, so its
output must be bit-identical to mmdx_attention_fwd's (same dropout mask from the same seed and
counter).  The backward recomputes P and the keep bits and takes rowsum(P o dP) as dO . O:
its gradients must match torch's autograd of the same masked, dropped-out attention, and
the P-saving backward's.  The bars are multiples of the 16-bit unit roundoff u (bf16 2^-8,
fp16 2^-11), relative to the output's / each gradient's own scale: the kernels round P (and
dS) to the 16-bit type before each product and the outputs once; the output within 2u of
torch's fp32, gradients within 4u of torch and of the P-saving kernels (measured on the test's
cases: 1.3u, 2.1u and 2.4u at most, gpurun_out r05).
"""
import pytest
import torch

from mmdx import _lib as L
from parity_util import rel_err

pytestmark = pytest.mark.gpu

U = {torch.bfloat16: 2.0 ** -8, torch.float16: 2.0 ** -11}   # unit roundoff of the 16-bit type


def _run(dev, dt, B, Ls, H, masked, pd, seed=77):
    g = torch.Generator().manual_seed(B * Ls + H + int(pd * 100))
    qkv = torch.randn(B, Ls, 3, H, 64, generator=g).to(dt).float()
    mask = None
    if masked:
        lens = torch.randint(1, Ls + 1, (B,), generator=g)
        mask = (torch.arange(Ls)[None] < lens[:, None]).long()
    do = torch.randn(B, Ls, H, 64, generator=g).to(dt).float()
    scale = 0.125
    dc = L.dtype_code(dt)
    qd = qkv.to(dev, dt).contiguous()
    dod = do.to(dev, dt).contiguous()
    md = mask.to(dev) if mask is not None else None
    mp = md.data_ptr() if md is not None else None
    # P-saving path
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    out0 = torch.empty(B, Ls, H, 64, dtype=dt, device=dev)
    probs = torch.empty(B, H, Ls, Ls, device=dev)
    L.call("mmdx_attention_fwd", dc, qd.data_ptr(), mp, B, Ls, H, scale, pd, seed,
           ctr.data_ptr(), out0.data_ptr(), probs.data_ptr(), L.stream())
    dq0 = torch.empty_like(qd)
    n0 = L.lib().mmdx_attention_workspace_size(dc, B, Ls, H)
    w0 = torch.empty(n0, dtype=torch.uint8, device=dev)
    L.call("mmdx_attention_bwd", dc, qd.data_ptr(), probs.data_ptr(), dod.data_ptr(), mp, B, Ls,
           H, scale, pd, dq0.data_ptr(), w0.data_ptr(), n0, L.stream())
    # flash-style path, same seed and counter value
    ctr.zero_()
    out1 = torch.empty_like(out0)
    lse = torch.empty(B, H, Ls, device=dev)
    rng = torch.empty(1, dtype=torch.int64, device=dev)
    L.call("mmdx_attention_fwd_lse", dc, qd.data_ptr(), mp, B, Ls, H, scale, pd, seed,
           ctr.data_ptr(), out1.data_ptr(), lse.data_ptr(), rng.data_ptr(), L.stream())
    dq1 = torch.full_like(qd, float("nan"))
    n1 = L.lib().mmdx_attention_lse_workspace_size(dc, B, Ls, H)
    w1 = torch.empty(n1, dtype=torch.uint8, device=dev)
    L.call("mmdx_attention_bwd_lse", dc, qd.data_ptr(), out1.data_ptr(), lse.data_ptr(),
           rng.data_ptr(), dod.data_ptr(), mp, B, Ls, H, scale, pd, dq1.data_ptr(),
           w1.data_ptr(), n1, L.stream())
    torch.cuda.synchronize()
    assert int(ctr.item()) == (1 if pd > 0 else 0)
    # torch reference with the kernel's own keep mask (sign of the saved probabilities)
    keep = ~torch.signbit(probs.cpu())
    qr = qkv.clone().requires_grad_(True)
    q, k, v = qr[:, :, 0], qr[:, :, 1], qr[:, :, 2]
    s = torch.einsum("blhd,bmhd->bhlm", q, k) * scale
    if mask is not None:
        s = s + (1.0 - mask[:, None, None, :].float()) * -1e30
    p = s.softmax(-1)
    o = torch.einsum("bhlm,bmhd->blhd", p * keep.float() / (1 - pd), v)
    o.backward(do)
    return dict(out0=out0, out1=out1, lse=lse, s=s.detach(), dq0=dq0, dq1=dq1, o=o.detach(),
                grad=qr.grad, qkv=qkv, do=do)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,Ls,H", [(2, 128, 12), (3, 37, 2), (2, 197, 4), (1, 256, 1),
                                    (1, 1, 3), (4, 129, 6)])
@pytest.mark.parametrize("masked,pd", [(False, 0.0), (True, 0.0), (True, 0.1)])
def test_flash_attention(dev, dt, B, Ls, H, masked, pd):
    r = _run(dev, dt, B, Ls, H, masked, pd)
    u = U[dt]
    assert torch.equal(r["out1"], r["out0"]), "forward output differs from the P-saving kernel"
    eo = rel_err(r["out1"], r["o"])
    print(f"  out err {eo / u:.2f}u", end="")
    assert eo <= 2 * u, eo
    ref_lse = torch.logsumexp(r["s"], -1)
    assert (r["lse"].cpu() - ref_lse).abs().max().item() <= 1e-3 * max(1.0, ref_lse.abs().max())
    assert torch.isfinite(r["dq1"]).all()
    if Ls == 1:
        # one key: the exact dQ and dK are 0 (constant softmax).  The flash backward's row term
        # D = dO . O uses the 16-bit output, so dS = P (dP - D) is the rounding of O alone:
        # |dS| <= 2^-7 sum_d |dO_d O_d| (and dQ = scale dS K, dK = scale dS Q)
        o16 = r["out1"].float().cpu()
        do16 = r["do"]
        ds_max = 2.0 ** -7 * (do16.abs() * o16.abs()).sum(-1, keepdim=True)   # [B, L, H, 1]
        q, k = r["qkv"][:, :, 0], r["qkv"][:, :, 1]
        d = r["dq1"].float().cpu()
        assert (d[:, :, 0].abs() <= 0.125 * ds_max * k.abs() + 1e-6).all(), "dQ at L = 1"
        assert (d[:, :, 1].abs() <= 0.125 * ds_max * q.abs() + 1e-6).all(), "dK at L = 1"
        assert _err(r["dq1"], r["grad"], 2) <= 4 * u
        return
    for i, name in enumerate("qkv"):
        e = _err(r["dq1"], r["grad"], i)
        e2 = _err(r["dq1"], r["dq0"].float().cpu(), i)
        print(f" d{name} {e / u:.2f}u / {e2 / u:.2f}u", end="")
        assert e <= 4 * u, f"d{name} vs torch {e}"
        assert e2 <= 4 * u, f"d{name} vs P-saving kernels {e2}"


def _err(got, ref, i):
    """max |error| of gradient i relative to its own scale, floored at 5 % of the largest of
    the three (dQ and dK vanish exactly at L = 1, where the softmax is constant)."""
    got = got[:, :, i].float().cpu()
    ref_all = ref.float().cpu()
    ref = ref_all[:, :, i]
    den = max(ref.abs().max().item(), 0.05 * ref_all.abs().max().item(), 1e-30)
    return (got - ref).abs().max().item() / den


def test_flash_attention_vit_bert_shapes(dev):
    """The benched C5 geometries (ViT-B/16 L 197, BERT-base L 128 with dropout 0.1, 12
    heads, fp16) at a reduced batch."""
    for Ls, masked, pd in ((197, False, 0.0), (128, True, 0.1)):
        r = _run(dev, torch.float16, 4, Ls, 12, masked, pd)
        assert torch.equal(r["out1"], r["out0"])
        assert rel_err(r["out1"], r["o"]) <= 2 * U[torch.float16]
        for i in range(3):
            assert _err(r["dq1"], r["grad"], i) <= 4 * U[torch.float16]
