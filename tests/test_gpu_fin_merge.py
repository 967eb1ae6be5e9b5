"""The 16-to-1 merge of finalize row partials (unetseg_fin_merge_rows, ops._merge_rows) against the finalizes
run on the unmerged rows: BatchNorm2d statistics (Chan's merge of (sum, M2) rows, reference
model/resnet_backbone.py:64-70 BatchNorm2d in train mode) and the plain sums of the backward post-op
partials.  The merged rows are rounded to fp32 once, so the outputs agree to fp32 rounding of the
partial sums (rtol 1e-5), not bit for bit.  Row counts: the bench's 512^2 B=8 (8192 rows of 256 pixels),
2048, and a ragged 601 rows whose last tile holds 37 pixels."""
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


def _stats_rows(G, C, tile, M, g):
    """plausible (sum, M2) rows: per-row counts, means around 0.3, variances around 1.2"""
    cnt = torch.full((G,), float(tile), device=DEV)
    cnt[-1] = float(M - (G - 1) * tile)
    mean = 0.3 + 0.1 * torch.randn(G, C, device=DEV, generator=g)
    var = 1.2 * torch.rand(G, C, device=DEV, generator=g) + 0.1
    part = torch.empty(G, 2, C, device=DEV)
    part[:, 0] = mean * cnt[:, None]
    part[:, 1] = var * cnt[:, None]
    return part


@pytest.mark.parametrize("G,C,tile,last", [(8192, 64, 256, 256), (2048, 128, 256, 256), (601, 96, 256, 37)])
def test_merge_bn_finalize(G, C, tile, last):
    from unetseg_hip.lib import lib
    st = torch.cuda.current_stream().cuda_stream
    M = (G - 1) * tile + last
    g = torch.Generator(device=DEV).manual_seed(G + C)
    part = _stats_rows(G, C, tile, M, g)
    gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    outs = []
    for merge in (False, True):
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        nbt = torch.zeros(1, dtype=torch.long, device=DEV)
        o = [torch.empty(C, device=DEV) for _ in range(4)]
        p, rows, t = part, G, tile
        if merge:
            rows = (G + 15) // 16
            p = torch.empty(rows, 2, C, device=DEV)
            lib.fin_merge_rows(part.data_ptr(), C, G, M, tile, 2, p.data_ptr(), st)
            t = tile * 16
        lib.bn_finalize(p.data_ptr(), C, rows, M, t, gamma.data_ptr(), beta.data_ptr(), rm.data_ptr(), rv.data_ptr(),
                        nbt.data_ptr(), 0.1, 1e-5, *(x.data_ptr() for x in o), st)
        torch.cuda.synchronize()
        outs.append(torch.stack(o + [rm, rv]))
    torch.testing.assert_close(outs[1], outs[0], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("G,C,nq", [(8192, 64, 2), (2048, 256, 3), (601, 96, 2)])
def test_merge_plain_sums(G, C, nq):
    from unetseg_hip.lib import lib
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=DEV).manual_seed(G * 3 + C)
    part = torch.randn(G, nq, C, device=DEV, generator=g)
    rows = (G + 15) // 16
    merged = torch.empty(rows, nq, C, device=DEV)
    lib.fin_merge_rows(part.data_ptr(), C, G, 0, 0, nq, merged.data_ptr(), st)
    torch.cuda.synchronize()
    ref = torch.nn.functional.pad(part.double(), (0, 0, 0, 0, 0, rows * 16 - G)).view(rows, 16, nq, C).sum(1)
    torch.testing.assert_close(merged.double(), ref, rtol=1e-6, atol=1e-5)
    # and through a finalize: the column sums of both forms agree to fp32 rounding
    out0, out1 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    if nq == 2:
        lib.colsum_rows(part.data_ptr(), C, G, 1, out0.data_ptr(), 0, st)
        lib.colsum_rows(merged.data_ptr(), C, rows, 1, out1.data_ptr(), 0, st)
        torch.cuda.synchronize()
        torch.testing.assert_close(out1, out0, rtol=1e-5, atol=1e-4)
