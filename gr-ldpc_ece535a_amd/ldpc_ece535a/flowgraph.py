"""A minimal single-threaded stand-in for the GNU Radio 3.7 scheduler.

GNU Radio is not installed in this environment, so the QA-style tests and
the CLI drive the blocks through this harness: it offers the pieces the
reference's QA tests use (gr.top_block, blocks.vector_source_*,
blocks.vector_sink_*, connect, run -- python/qa_ldpc_decoder_cb.py:45-55) and
calls each block's general_work the way the runtime does: with whatever input
has arrived (optionally in small, irregular chunks), a bounded output buffer,
unconsumed input carried over to the next call.
"""
import numpy as np


class vector_source_c:
    dtype = np.complex64

    def __init__(self, data, repeat=False):
        if repeat:
            raise NotImplementedError("repeat=True is not supported by the test harness")
        self._data = np.asarray(data, self.dtype)


class vector_source_b(vector_source_c):
    dtype = np.uint8


class vector_source_f(vector_source_c):
    dtype = np.float32


class vector_sink_b:
    dtype = np.uint8

    def __init__(self):
        self._parts = []

    def _push(self, items):
        if len(items):
            self._parts.append(np.asarray(items, self.dtype))

    def data(self):
        """Like GNU Radio: a tuple of the received items."""
        if not self._parts:
            return tuple()
        return tuple(np.concatenate(self._parts).tolist())

    def array(self):
        return np.concatenate(self._parts) if self._parts else np.zeros(0, self.dtype)


class vector_sink_c(vector_sink_b):
    dtype = np.complex64


class top_block:
    """Runs a linear chain source -> block* -> sink.

    chunk: None (whole input at once), an int, or a sequence of ints: how
    many source items become visible per scheduler round.  out_space: the
    output buffer (items) offered to each general_work call.
    """

    def __init__(self, name="top_block", chunk=None, out_space=8192):
        self.name = name
        self.chunk = chunk
        self.out_space = out_space
        self._edges = []

    def connect(self, *args):
        nodes = [a[0] if isinstance(a, tuple) else a for a in args]
        for a, b in zip(nodes[:-1], nodes[1:]):
            self._edges.append((a, b))

    def _chain(self):
        nexts = dict(self._edges)
        heads = [a for a, _ in self._edges if a not in set(b for _, b in self._edges)]
        if len(heads) != 1:
            raise ValueError("top_block harness supports one linear chain")
        chain, node = [], heads[0]
        while node is not None:
            chain.append(node)
            node = nexts.get(node)
        return chain

    def run(self):
        chain = self._chain()
        src, blocks, sink = chain[0], chain[1:-1], chain[-1]
        data = src._data
        if self.chunk is None:
            sizes = [len(data)]
        elif isinstance(self.chunk, int):
            sizes = [self.chunk] * (len(data) // self.chunk + 1)
        else:
            sizes = list(self.chunk)
        bufs = [np.zeros(0, src.dtype)] + [None] * len(blocks)
        pos = 0
        rounds = 0
        while True:
            progress = False
            if pos < len(data):
                n = sizes[rounds] if rounds < len(sizes) else len(data) - pos
                rounds += 1
                bufs[0] = np.concatenate([bufs[0], data[pos:pos + n]])
                pos += n
                progress = True
            for k, blk in enumerate(blocks):
                while True:
                    out, used = blk.general_work(self.out_space, bufs[k])
                    if used:
                        bufs[k] = bufs[k][used:]
                    if len(out):
                        if k + 1 < len(blocks):
                            nxt = bufs[k + 1]
                            bufs[k + 1] = out if nxt is None else np.concatenate([nxt, out])
                        else:
                            sink._push(out)
                    if used or len(out):
                        progress = True
                    else:
                        break
            if not progress and pos >= len(data):
                break
            if pos >= len(data) and not progress:
                break
            if not progress:
                continue

    def start(self):
        self.run()

    def wait(self):
        pass
