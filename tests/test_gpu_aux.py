"""GPU: device encoder, channel, error counts and the BER sweep (SURVEY
8(f) rows 2-3) against the host encoders and numpy."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _dev(a):
    """Device copy; callers keep the returned tensor alive while it is used
    (a temporary's storage goes back to the caching allocator at once)."""
    import torch
    t = torch.from_numpy(np.ascontiguousarray(a)).cuda(0)
    torch.cuda.synchronize()
    return t


@pytest.mark.parametrize("name", ["decoder_h", "qa_h", "hData1", "hData5"])
def test_encode_device_matches_host_encoder(golden, name):
    """ldpc_encode_device == makeParityCheck (the host GF(2) encoder pinned
    by the reference's encoder KAT) on the reordered H."""
    import torch
    import ldpc_ece535a as L
    H = golden("reference_data.npz")[name]
    d = L.Decoder(H)
    if d.N != 2 * d.M:
        pytest.skip("host encoder needs N == 2M")
    rng = np.random.default_rng(3)
    data = rng.integers(0, 2, (333, d.K), dtype=np.uint8)
    cw = torch.empty((333, d.N), dtype=torch.uint8, device="cuda:0")
    x = _dev(data)
    d.encode_device(x.data_ptr(), 333, cw.data_ptr())
    d.synchronize()
    assert (cw.cpu().numpy() == L.encode(d.H, data)).all()


def test_encode_device_kat_8x16(golden):
    import torch
    import ldpc_ece535a as L
    ref = golden("reference_data.npz")
    d = L.Decoder(ref["qa_h"])
    data = np.unpackbits(ref["kat_data"]).reshape(8, 8)
    cw = torch.empty((8, 16), dtype=torch.uint8, device="cuda:0")
    x = _dev(data)
    d.encode_device(x.data_ptr(), 8, cw.data_ptr())
    d.synchronize()
    assert ((2 * cw.cpu().numpy()[:, :8].astype(int) - 1) == ref["kat_mod_check"]).all()


def test_encode_device_ira_matches_host():
    import torch
    import ldpc_ece535a as L
    from ldpc_ece535a import codes
    csr = codes.dvbs2_like(0)
    d = L.Decoder(csr=csr)
    rng = np.random.default_rng(4)
    data = rng.integers(0, 2, (37, d.K), dtype=np.uint8)
    cw = torch.empty((37, d.N), dtype=torch.uint8, device="cuda:0")
    x = _dev(data)
    d.encode_device(x.data_ptr(), 37, cw.data_ptr())
    d.synchronize()
    got = cw.cpu().numpy()
    assert (got == codes.ira_encode(csr, data)).all()
    assert (codes.syndrome_weight(csr, got[:4]) == 0).all()


def test_encode_device_rejects_non_staircase_large_code():
    import ldpc_ece535a as L
    M, N = 300, 600
    rp = np.arange(0, 3 * M + 1, 3, dtype=np.int32)
    ci = np.array([[j, (j + 7) % M, M + j] for j in range(M)], np.int32)
    ci.sort(axis=1)
    d = L.Decoder(csr=(M, N, rp, ci.reshape(-1)))
    import torch
    x = torch.zeros((1, N - M), dtype=torch.uint8, device="cuda:0")
    y = torch.zeros((1, N), dtype=torch.uint8, device="cuda:0")
    with pytest.raises(L.LdpcError, match="staircase"):
        d.encode_device(x.data_ptr(), 1, y.data_ptr())


def test_random_bits_and_awgn_statistics():
    import torch
    from ldpc_ece535a import _capi
    n = 1 << 22
    bits = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    _capi.random_bits(bits.data_ptr(), n, 123)
    torch.cuda.synchronize()
    b = bits.cpu().numpy()
    assert set(np.unique(b)) <= {0, 1} and abs(b.mean() - 0.5) < 2e-3
    again = torch.empty_like(bits)
    _capi.random_bits(again.data_ptr(), n, 123)
    torch.cuda.synchronize()
    assert (again.cpu().numpy() == b).all()  # reproducible
    out = torch.empty(n, dtype=torch.float32, device="cuda:0")
    sigma = 0.7
    _capi.bpsk_awgn(bits.data_ptr(), n, sigma, 9, out.data_ptr())
    torch.cuda.synchronize()
    noise = out.cpu().numpy().astype(np.float64) - (2.0 * b - 1.0)
    assert abs(noise.mean()) < 2e-3 and abs(noise.std() - sigma) < 2e-3
    assert abs(((noise / sigma) ** 4).mean() - 3.0) < 0.05  # Gaussian kurtosis


def test_count_bit_errors():
    import torch
    from ldpc_ece535a import _capi
    rng = np.random.default_rng(5)
    a = rng.integers(0, 2, (77, 1000), dtype=np.uint8)
    b = a.copy()
    flips = rng.random(a.shape) < 0.03
    b[flips] ^= 1
    cnt = torch.empty(77, dtype=torch.int32, device="cuda:0")
    da, db = _dev(a), _dev(b)
    _capi.count_bit_errors(da.data_ptr(), db.data_ptr(), 1000, 77, cnt.data_ptr())
    torch.cuda.synchronize()
    assert (cnt.cpu().numpy() == flips.sum(axis=1)).all()


def test_ber_sweep_shape_and_monotone():
    """The reference program's sweep on the GPU: every curve falls with
    Eb/N0; the hard decision follows Q(1/sigma) (the reference's convention
    has no rate factor: 10 dB is sigma = 0.316, BER ~ 7.9e-4); sum-product
    beats it once decoding works and is error-free at 10 dB."""
    import math
    from ldpc_ece535a import ber
    grid = [-2.0, 2.0, 6.0, 10.0]
    res = ber.sweep(ebn0=grid, frames=4000, iterations=5, seed=1)
    for name, _ in ber.METHODS:
        b = res[name]["ber"]
        assert b[0] > b[1] > b[2] >= b[3]
        assert len(res[name]["fer"]) == 4
    q = [0.5 * math.erfc(1.0 / ber.sigma_of(db) / math.sqrt(2.0)) for db in grid]
    for got, want in zip(res["BPSK"]["ber"], q):
        assert abs(got - want) < 4 * math.sqrt(want / (4000 * 64)) + 1e-5
    assert res["SumProduct"]["ber"][2] < res["BPSK"]["ber"][2]
    assert res["SumProduct"]["ber"][3] == 0.0 and res["SumProduct"]["fer"][3] == 0
    txt = ber.octave(grid, res)
    assert txt.startswith("EbN0=[-2 2 6 10 ];") and "legend('BPSK', 'BitFlip'" in txt
