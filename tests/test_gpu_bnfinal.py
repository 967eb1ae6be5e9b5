"""GPU: the BN finalize reductions over row partials [G][2][C] (unetseg_bn_finalize,
unetseg_bn_bwd_finalize_rows) against fp64 torch: up to 16k row tiles (the 512^2 layers of
unet_plain / attention_unet), channel counts 1..2048 that are not all multiples of 64, and a ragged
last row tile."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _lib():
    from unetseg_hip.lib import lib
    return lib


@pytest.mark.parametrize("M,C,tile", [(300_001, 1, 128), (300_001, 96, 256), (65_536, 200, 128), (4_096, 2048, 128),
                                      (2_000, 64, 256), (4_194_304, 64, 256)])
def test_bn_finalize_rows(M, C, tile):
    lib = _lib()
    g = torch.Generator(device=DEV).manual_seed(M + C)
    x = torch.randn(M, C, generator=g, device=DEV, dtype=torch.float64) * 2.0 + 0.7
    G = -(-M // tile)
    part = torch.empty(G, 2, C, device=DEV, dtype=torch.float32)
    for g0 in range(0, G, 4096):  # per-row-tile (sum, M2 about the tile mean), as the conv epilogues
        rows = x[g0 * tile:min(M, (g0 + 4096) * tile)]
        n = rows.shape[0]
        full = n // tile
        sums, m2 = [], []
        if full:
            t = rows[:full * tile].view(full, tile, C)
            sums.append(t.sum(1))
            m2.append(((t - t.mean(1, keepdim=True)) ** 2).sum(1))
        if n % tile:
            t = rows[full * tile:]
            sums.append(t.sum(0, keepdim=True))
            m2.append(((t - t.mean(0, keepdim=True)) ** 2).sum(0, keepdim=True))
        part[g0:g0 + len(torch.cat(sums))] = torch.stack([torch.cat(sums), torch.cat(m2)], 1).float()
    gamma = torch.rand(C, generator=g, device=DEV) + 0.5
    beta = torch.randn(C, generator=g, device=DEV)
    rm = torch.randn(C, generator=g, device=DEV)
    rv = torch.rand(C, generator=g, device=DEV) + 0.5
    rm0, rv0 = rm.clone(), rv.clone()
    nbt = torch.zeros(1, dtype=torch.int64, device=DEV)
    mean, inv, sc, sh = (torch.empty(C, device=DEV) for _ in range(4))
    st = torch.cuda.current_stream().cuda_stream
    P = lambda t: t.data_ptr()  # noqa: E731
    lib.bn_finalize(P(part), C, G, M, tile, P(gamma), P(beta), P(rm), P(rv), P(nbt), 0.1, 1e-5, P(mean), P(inv),
                    P(sc), P(sh), st)
    torch.cuda.synchronize()
    # reference from the fp32-rounded partials (what the kernel sees), merged in fp64
    mu = x.mean(0)
    var = x.var(0, unbiased=False)
    torch.testing.assert_close(mean.double(), mu, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(inv.double(), 1 / torch.sqrt(var + 1e-5), rtol=1e-5, atol=0)
    torch.testing.assert_close(sc.double(), gamma.double() / torch.sqrt(var + 1e-5), rtol=1e-5, atol=0)
    torch.testing.assert_close(sh.double(), beta.double() - mu * gamma.double() / torch.sqrt(var + 1e-5),
                               rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(rm.double(), 0.9 * rm0.double() + 0.1 * mu, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rv.double(), 0.9 * rv0.double() + 0.1 * x.var(0, unbiased=True), rtol=1e-5, atol=1e-6)
    assert int(nbt) == 1


@pytest.mark.parametrize("G,C", [(2_345, 1), (2_345, 96), (20_000, 64), (64, 2048), (3, 200)])
def test_bn_bwd_finalize_rows(G, C):
    lib = _lib()
    g = torch.Generator(device=DEV).manual_seed(G * 7 + C)
    part = torch.randn(G, 2, C, generator=g, device=DEV)
    ref = part.double().sum(0)
    g1 = torch.rand(C, generator=g, device=DEV) + 0.5
    inv1 = torch.rand(C, generator=g, device=DEV) + 0.5
    dg = torch.randn(C, generator=g, device=DEV)
    db = torch.randn(C, generator=g, device=DEV)
    dg0, db0 = dg.clone(), db.clone()
    coef = torch.zeros(6, C, device=DEV)
    M = G * 128
    P = lambda t: t.data_ptr()  # noqa: E731
    lib.bn_bwd_finalize_rows(P(part), C, G, M, P(g1), P(inv1), P(dg), P(db), P(coef),
                             torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    torch.testing.assert_close(db.double(), db0.double() + ref[0], rtol=1e-6, atol=1e-5)
    torch.testing.assert_close(dg.double(), dg0.double() + ref[1], rtol=1e-6, atol=1e-5)
    torch.testing.assert_close(coef[0], g1 * inv1)
    torch.testing.assert_close(coef[1].double(), ref[0] / M, rtol=1e-6, atol=1e-9)
    torch.testing.assert_close(coef[2].double(), ref[1] / M, rtol=1e-6, atol=1e-9)
