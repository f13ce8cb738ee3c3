"""Concurrent launches of one context on several HIP streams.

ldpc_decode_device takes the caller's stream.  Small-code launches on
different streams run concurrently, each on its own frame-queue counter
(ldpc_kernels.hpp DecodeArgs::ticket); large-code launches share one
workspace and are ordered across streams by the context.  Interleaved
launches on two streams, plus a synchronous host-buffer decode on the
context's own stream in between, must give exactly the single-stream results.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frames(Hr, B, db, seed):
    import ldpc_ece535a as L
    rng = np.random.Generator(np.random.PCG64(seed))
    x = 2.0 * L.encode(Hr, rng.integers(0, 2, size=(B, Hr.shape[1] - Hr.shape[0]),
                                        dtype=np.uint8)) - 1.0
    return (x + np.sqrt(10 ** (-db / 10)) * rng.standard_normal(x.shape)).astype(np.float32)


@pytest.mark.parametrize("method", [1, 0])
@pytest.mark.parametrize("graph", [False, True])
def test_interleaved_streams(graph, method):
    """method 0 on the large-code path is the compressed-message min-sum
    pipeline, whose passes are all enqueued without a host round trip."""
    import torch
    import ldpc_ece535a as L
    dec = L.Decoder(force_graph=graph)
    B = 4096 if not graph else 512
    ys = [_frames(dec.H, B, db, 900 + k) for k, db in enumerate((2.0, 0.0, 3.0))]
    refs = [dec.decode(y, method=method, max_iters=50) for y in ys]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    d_in = [torch.from_numpy(y).cuda() for y in ys]
    launches = []
    for k in range(12):
        j = k % 3
        st = streams[k % 2]
        pk = torch.empty((B, dec.KB), dtype=torch.uint8, device="cuda")
        it = torch.empty(B, dtype=torch.int32, device="cuda")
        sy = torch.empty(B, dtype=torch.int32, device="cuda")
        with torch.cuda.stream(st):
            dec.decode_device(d_in[j].data_ptr(), B, pk.data_ptr(), method=method,
                              max_iters=50, d_iters=it.data_ptr(), d_synd=sy.data_ptr(),
                              stream=st.cuda_stream)
        launches.append((j, pk, it, sy))
        if k == 5:  # a host-buffer decode on the context's own stream meanwhile
            mid = dec.decode(ys[1], method=method, max_iters=50)
            assert (mid["packed"] == refs[1]["packed"]).all()
    torch.cuda.synchronize()
    for j, pk, it, sy in launches:
        assert (pk.cpu().numpy() == refs[j]["packed"]).all()
        assert (it.cpu().numpy() == refs[j]["iters"]).all()
        assert (sy.cpu().numpy() == refs[j]["synd"]).all()
    dec.close()


def test_many_streams_reuse_counters():
    """More streams than frame-queue counters: the context drains and starts
    its queues over; every launch still decodes its whole batch."""
    import torch
    import ldpc_ece535a as L
    dec = L.Decoder()
    y = _frames(dec.H, 3000, 2.0, 77)
    ref = dec.decode(y, method=0, max_iters=20)
    d_in = torch.from_numpy(y).cuda()
    # torch hands out streams from two pools of 32 (priority 0 and -1): with the
    # context's own stream (used by the reference decode above) that is 65
    # distinct streams, one more than the context's 64 counters
    for k in range(70):
        st = torch.cuda.Stream(priority=-1 if k % 2 else 0)
        pk = torch.empty((3000, dec.KB), dtype=torch.uint8, device="cuda")
        it = torch.empty(3000, dtype=torch.int32, device="cuda")
        with torch.cuda.stream(st):
            dec.decode_device(d_in.data_ptr(), 3000, pk.data_ptr(), method=0, max_iters=20,
                              d_iters=it.data_ptr(), stream=st.cuda_stream)
        st.synchronize()
        if k % 10 == 0 or k >= 63:
            assert (pk.cpu().numpy() == ref["packed"]).all(), k
            assert (it.cpu().numpy() == ref["iters"]).all(), k
    dec.close()
