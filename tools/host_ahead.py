"""How far the host runs ahead of the GPU in steady state (no syncs between steps).

    python tools/host_ahead.py
After enqueueing step k, reports whether step k-1's end event has completed, and the host time per
step (= GPU time per step when the host is throttled by the launch queue).
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    from model.model_factory import create_model
    from unetseg_hip.arena import FusedAdam
    from unetseg_hip.losses import binary_segmentation_loss
    from utils.synthetic import make_batch

    if os.environ.get("HA_STREAM", "1") == "1":  # bench.py's default: a created (non-legacy) stream
        torch.cuda.set_stream(torch.cuda.Stream())
    m = create_model("unet_resnet50", weights="", num_classes=2).cuda().train()
    m.compute_dtype = "bf16"
    # bench.py's optimizer: Adam + re-pack per gradient bucket during backward (HA_OVERLAP=0: after it)
    opt = FusedAdam(m, lr=1e-4, weight_decay=1e-4, overlap=os.environ.get("HA_OVERLAP", "1") == "1")
    x, y = make_batch(16, 512, seed=5)
    x, y = x.cuda(), y.cuda()

    def step():
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = binary_segmentation_loss(m(x), y, "lovasz_hinge")
        t_fwd = time.perf_counter()
        loss.backward()
        t_bwd = time.perf_counter()
        opt.step()
        return t_fwd, t_bwd

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    evs = []
    t_prev = time.perf_counter()
    for k in range(8):
        tf, tb = step()
        t = time.perf_counter()
        e = torch.cuda.Event()
        e.record()
        evs.append(e)
        done = [int(ev.query()) for ev in evs[-4:]]
        st = torch.cuda.memory_stats()
        print(f"step {k}: host {1e3 * (t - t_prev):6.2f} ms (fwd {1e3 * (tf - t_prev):5.2f}, bwd {1e3 * (tb - tf):5.2f}) "
              f"last-4 step events done: {done}  segments {st.get('segment.all.current', -1)} "
              f"alloc_retries {st.get('num_alloc_retries', -1)} hipMalloc {st.get('num_device_alloc', -1)}", flush=True)
        t_prev = t
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
