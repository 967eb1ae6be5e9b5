"""GPU: the loss / metric kernels at the benchmark's size against the CPU oracle.

The Lovasz kernel sorts each image's P hinge errors with a segmented LSD radix sort in
kTile = 4096-key tiles (csrc/loss.hip); P = 512^2 gives T = 64 tiles per image, whose cross-tile
digit histograms, scans and the Jaccard scan's carried counts are only exercised when T > 1.
Reference: model/unet_training.py:219-280 (per-image Lovasz, mean over images) restated in
oracle/ref_cpu.py:280-310, utils/train_and_eval.py:106-113 (z = o1 - o0).

Tie-free inputs make the sort order -- hence the per-pixel gradient -- unique:
z = (3k + 1) / 2^15 - 4 over a random permutation of k; two errors 1 - z_i and 1 + z_j can only be
equal if 3(k_i + k_j) + 2 = 2^18, which has no integer solution.  With ties only the loss VALUE is
order-independent, so the tied cases compare the value alone.
Tolerances: loss 2e-6 relative, gradient 1e-5 of its max (fp32 scans vs the oracle's fp32 cumsum).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from unetseg_hip import load
    load()


def _tie_free(B, H, W, g):
    P = H * W
    assert 3 * P + 1 < (1 << 24)
    z = torch.empty(B, P)
    for b in range(B):
        k = torch.randperm(P, generator=g).double()
        z[b] = ((3 * k + 1) / 32768.0 - 4.0).float()
    return z.view(B, H, W)


def _two(z):
    return torch.stack([torch.zeros_like(z), z], 1)


@pytest.mark.parametrize("B,H,W", [(16, 512, 512), (3, 300, 300), (2, 97, 131), (1, 1024, 1056)])
def test_lovasz_multitile_tie_free(B, H, W):
    """loss and dloss/dlogits at T = ceil(P / 4096) = 64 / 22 / 4 / 264 tiles per image (past 128 tiles the
    radix scan keeps its runs in memory instead of registers)"""
    from oracle import ref_cpu
    from unetseg_hip import losses
    g = torch.Generator().manual_seed(B * 7 + H)
    z = _tie_free(B, H, W, g)
    tgt = (torch.rand(B, H, W, generator=g) < 0.3).long()
    o = _two(z).requires_grad_(True)
    ref = ref_cpu.binary_segmentation_loss(o, tgt, "lovasz_hinge")
    ref.backward()
    od = _two(z).to(DEV).requires_grad_(True)
    loss = losses.binary_segmentation_loss(od, tgt.to(DEV), "lovasz_hinge")
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - ref.item()) <= 2e-6 * abs(ref.item()), (loss.item(), ref.item())
    gd, gr = od.grad.cpu().double(), o.grad.double()
    err = (gd - gr).abs().max().item()
    assert err <= 1e-5 * gr.abs().max().item(), err


@pytest.mark.parametrize("B,H,W,levels", [(16, 512, 512, 5), (4, 300, 300, 0)])
def test_lovasz_multitile_ties_value(B, H, W, levels):
    """heavy ties (logits on a few levels, or bf16-rounded): loss value only"""
    from oracle import ref_cpu
    from unetseg_hip import losses
    g = torch.Generator().manual_seed(B + levels)
    if levels:
        z = (torch.randint(0, levels, (B, H, W), generator=g).float() - levels // 2) * 0.5
    else:
        z = (torch.randn(B, H, W, generator=g) * 2).to(torch.bfloat16).float()
    tgt = (torch.rand(B, H, W, generator=g) < 0.4).long()
    ref = ref_cpu.binary_segmentation_loss(_two(z), tgt, "lovasz_hinge")
    loss = losses.binary_segmentation_loss(_two(z).to(DEV), tgt.to(DEV), "lovasz_hinge")
    assert abs(loss.item() - ref.item()) <= 1e-5 * abs(ref.item()), (loss.item(), ref.item())


def test_lovasz_all_one_class():
    """images with no foreground / all foreground (the Jaccard denominator's edge cases)"""
    from oracle import ref_cpu
    from unetseg_hip import losses
    g = torch.Generator().manual_seed(3)
    z = _tie_free(2, 128, 96, g)
    tgt = torch.zeros(2, 128, 96, dtype=torch.long)
    tgt[1] = 1
    o = _two(z).requires_grad_(True)
    ref = ref_cpu.binary_segmentation_loss(o, tgt, "lovasz_hinge")
    ref.backward()
    od = _two(z).to(DEV).requires_grad_(True)
    loss = losses.binary_segmentation_loss(od, tgt.to(DEV), "lovasz_hinge")
    loss.backward()
    assert abs(loss.item() - ref.item()) <= 2e-6 * max(1.0, abs(ref.item()))
    assert (od.grad.cpu().double() - o.grad.double()).abs().max().item() <= 1e-5 * max(1e-12, o.grad.abs().max().item())


def test_bce_and_confusion_bench_size():
    """BCE-with-logits (model/unet_training.py:205-216) and the confusion counts
    (utils/train_and_eval.py:116-137, argmax tie -> class 0) over B=16 x 512^2"""
    from oracle import ref_cpu
    from unetseg_hip import losses
    g = torch.Generator().manual_seed(11)
    out = torch.randn(16, 2, 512, 512, generator=g) * 3
    out[:, 1, :4] = out[:, 0, :4]  # exact ties -> background
    tgt = (torch.rand(16, 512, 512, generator=g) < 0.3).long()
    o = out.clone().requires_grad_(True)
    ref = ref_cpu.binary_segmentation_loss(o, tgt, "bce")
    ref.backward()
    od = out.to(DEV).requires_grad_(True)
    loss = losses.binary_segmentation_loss(od, tgt.to(DEV), "bce")
    loss.backward()
    assert abs(loss.item() - ref.item()) <= 1e-5 * abs(ref.item())
    assert (od.grad.cpu() - o.grad).abs().max().item() <= 1e-5 * o.grad.abs().max().item()
    conf = losses.binary_confusion(out.to(DEV), tgt.to(DEV)).cpu().tolist()
    assert conf == [int(v) for v in ref_cpu.binary_confusion(out, tgt)]
