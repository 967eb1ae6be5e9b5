"""GPU: run-to-run bitwise determinism: the same forward + Lovasz + backward, repeated
in one process with the caching allocator handing out different blocks each time and the weight
gradients on their side stream, gives bit-identical gradients.  Every reduction here is
fixed-order (split-K slabs reduced in slab order, BN / loss partials merged in fp64 in a fixed
order, stable radix sort), so any difference is a race."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("name,dt,size,batch", [("unet_resnet50", "bf16", 128, 4), ("attention_unet", "bf16", 64, 2),
                                                ("unet_plain", "fp32", 64, 2), ("dualdense_unet", "bf16", 64, 2)])
def test_gradients_bitwise_repeatable(name, dt, size, batch):
    from model.model_factory import build_model
    from unetseg_hip import losses
    from utils.synthetic import make_batch

    torch.manual_seed(0)
    m = build_model(name, num_classes=2).to(DEV).train()
    m.compute_dtype = dt
    x, y = make_batch(batch, size, seed=21)
    x, y = x.to(DEV), y.to(DEV)
    ref, junk = None, []
    for it in range(4):
        for p in m.parameters():
            p.grad = None
        loss = losses.binary_segmentation_loss(m(x), y, "lovasz_hinge")
        loss.backward()
        torch.cuda.synchronize()
        g = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
        if ref is None:
            ref = (loss.detach().clone(), g)
        else:
            assert torch.equal(loss, ref[0]), it
            diff = [k for k in g if not torch.equal(g[k], ref[1][k])]
            assert not diff, f"iteration {it}: {len(diff)} gradients differ, e.g. {diff[:3]}"
        junk = junk[len(junk) // 2:] + [torch.empty((it + 1) * 1234567, dtype=torch.uint8, device=DEV)]
