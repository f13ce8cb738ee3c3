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


@pytest.mark.parametrize("extra", [0, 1, 3])
def test_ctx_streams_run_concurrently(extra):
    """ldpc_ctx_streams' set runs its launches side by side whatever streams
    the process made before (in the suite's own crowded process;
    profiles/round5/inflight_bimodal.txt: a set with two streams on one
    hardware queue measured 0.72x).  Checked with device clocks, not wall
    time: a 0.2 ms spin on each of two streams, and the two spins' intervals
    must intersect (LDPC_TEST_STREAM_OVERLAP); the same stream twice must
    not.  The in-flight outputs equal the one-stream run's."""
    import torch
    import ldpc_ece535a as L
    from ldpc_ece535a._capi import TEST_STREAM_OVERLAP
    keep = [torch.cuda.Stream() for _ in range(extra)]  # queue history
    for st in keep:
        with torch.cuda.stream(st):
            torch.ones(16, device="cuda").sum()
    torch.cuda.synchronize()
    dec = L.Decoder()
    dec.set_launch_mode(1)
    hs = dec.streams(4)
    # this process has made dozens of streams by now (the suite's earlier
    # tests), and the GPU's hardware queue slots are shared by every queue of
    # every process: the set may hold fewer than four distinct streams, handed
    # out again in turn (include/ldpc_hip.h); those it holds must run side by
    # side.
    u = sorted(set(hs), key=hs.index)
    assert dec.streams_distinct == len(u) >= 2
    assert dec.test_hook(TEST_STREAM_OVERLAP, 0) == 0  # one stream: one after the other
    for i in range(len(u)):
        for j in range(len(u)):
            if i != j:
                assert dec.test_hook(TEST_STREAM_OVERLAP, (i << 8) | j) == 1, (i, j)
    B = 4096
    ys = [torch.from_numpy(_frames(dec.H, B, 2.0, 40 + j)).cuda() for j in range(4)]
    outs = [torch.empty((B, dec.KB), dtype=torch.uint8, device="cuda") for _ in range(4)]
    its = [torch.empty(B, dtype=torch.int32, device="cuda") for _ in range(4)]

    def run(streams):
        for d, st in enumerate(streams):
            dec.decode_device(ys[d].data_ptr(), B, outs[d].data_ptr(), method=1,
                              max_iters=50, d_iters=its[d].data_ptr(), stream=st)
        torch.cuda.synchronize()

    run([hs[0]] * 4)  # the four batches one after another on one stream
    one = [(outs[d].cpu().numpy().copy(), its[d].cpu().numpy().copy()) for d in range(4)]
    run(hs)
    for d in range(4):
        assert (outs[d].cpu().numpy() == one[d][0]).all()
        assert (its[d].cpu().numpy() == one[d][1]).all()
    dec.close()
