"""Debug a step plan against eager steps: which tensors differ after the first replay (names)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402

from test_gpu_plan import _setup, _state  # noqa: E402


def main():
    from unetseg_hip.plan import StepPlan
    from utils.synthetic import make_batch
    name, batch, size, loss_name = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    torch.cuda.set_stream(torch.cuda.Stream("cuda"))
    data = []
    for i in range(2):
        x, y, c = make_batch(batch, size, seed=1234 + i, with_cls=True)
        data.append((x.cuda(), y.cuda(), c.cuda()))
    ma, oa, sa = _setup(name, batch, size, loss_name)
    ref = [_state(ma, oa, sa(*data[i % 2])) for i in range(3)]
    mb, ob, sb = _setup(name, batch, size, loss_name)
    log = []
    orig = ob._bucket_update

    def upd(i, s, e, stream):
        log.append((i, s, e, ob._step, stream is not None))
        return orig(i, s, e, stream)
    bk = mb._buckets
    bk.actions[bk.actions.index(orig)] = upd
    got = [_state(mb, ob, sb(*data[0]))]
    print("eager0 updates", log); log.clear()
    plan = StepPlan({"x": data[1][0], "y": data[1][1], "c": data[1][2]})
    got.append(_state(mb, ob, plan.record(lambda: sb(*data[1]))))
    print("record updates", log); log.clear()
    got.append(_state(mb, ob, plan.replay(x=data[0][0], y=data[0][1], c=data[0][2])))
    print("replay updates", log); log.clear()
    torch.cuda.synchronize()
    print(plan.stats())
    for k, call in enumerate(plan.calls):
        if call[0] != "c":
            print(k, call[0], getattr(call[1], "__name__", call[1]))
    names = {}
    for n, p in mb.named_parameters():
        names[n] = mb.flat_slice(p)
    for step in range(3):
        a, b = ref[step], got[step]
        for lab, u, v in zip(("params", "grads", "m", "v"), a[:4], b[:4]):
            d = (u != v)
            if d.any():
                bad = [n for n, (o, l) in names.items() if d[o:o + l].any()]
                print(f"step {step} {lab}: {len(bad)} tensors differ: {bad[:12]}")
        print(f"step {step} bufs equal {torch.equal(a[4], b[4])} loss {a[5].item()} {b[5].item()} step {a[6]} {b[6]}")


if __name__ == "__main__":
    main()
