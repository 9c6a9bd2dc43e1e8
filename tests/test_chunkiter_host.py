"""Host side of RabinChunkIter (rabin.rs:110-191's read loop) without a GPU:
the device stream is replaced by a stand-in that cuts every 700001 bytes and
hands cuts out one piece late (as rcdc_stream_feed may), so the block reuse,
the chunks that span reads and blocks and the block reuse across iterators
are checked against plain byte slicing.  The cut points themselves are the GPU tests'."""
import gc
import io
import random

import numpy as np
import pytest

from rustic_core_amd import chunker as C

K = 700001


class _FakeStream:
    def __init__(self, ctx):
        self.n, self.pending, self.closed = 0, [], False

    def feed(self, data, fin):
        a = self.n
        self.n += len(data)
        new = [c for c in range((a // K + 1) * K, self.n, K)]
        out, self.pending = self.pending, new
        if fin:
            out = out + self.pending + ([self.n] if self.n else [])
            self.pending = []
        return np.array(out, np.uint64)

    def close(self):
        self.closed = True


class _Ctx:
    avg, min_size, max_size = 1 << 20, 512 << 10, 8 << 20


class _Short(io.RawIOBase):
    """readinto returns 1..k bytes per call."""

    def __init__(self, data, k, seed):
        self._b, self._k, self._r = io.BytesIO(data), k, random.Random(seed)

    def readable(self):
        return True

    def readinto(self, mv):
        b = self._b.read(min(len(mv), self._r.randint(1, self._k)))
        mv[:len(b)] = b
        return len(b)


@pytest.fixture
def fake(monkeypatch):
    monkeypatch.setattr(C, "_Stream", _FakeStream)
    monkeypatch.setattr(C, "check_rabin_params", lambda *a: None)


@pytest.mark.parametrize("ahead", ["1", "0"])
@pytest.mark.parametrize("size", [0, 1, K, 3 << 20, 16 << 20, (16 << 20) + 3, 70 << 20])
@pytest.mark.parametrize("kind", ["bytesio", "short", "buffered"])
def test_chunks_are_the_bytes_between_cuts(fake, monkeypatch, size, kind, ahead):
    """Also with the read ahead (a reader thread once a read fills a whole
    block) on and off (RCDC_READ_AHEAD)."""
    monkeypatch.setenv("RCDC_READ_AHEAD", ahead)
    data = np.random.default_rng(size).integers(0, 256, size, dtype=np.uint8).tobytes()
    reader = {"bytesio": lambda: io.BytesIO(data),
              "short": lambda: _Short(data, 3 << 20, size),
              "buffered": lambda: io.BufferedReader(io.BytesIO(data))}[kind]()
    it = C.RabinChunkIter(_Ctx(), reader, size)
    chunks = list(it)
    assert b"".join(chunks) == data
    want = list(range(K, size, K)) + ([size] if size else [])
    assert np.cumsum([len(c) for c in chunks]).tolist() == want
    assert it._stream.closed
    assert it._threaded == (ahead == "1" and kind != "short" and size >= C.READ_SIZE)
    assert list(it) == [] and it.size_hint == 0


def test_blocks_are_reused(fake):
    """Spent blocks go back to the pool and the next file reads into them."""
    C._POOL.clear()
    list(C.RabinChunkIter(_Ctx(), io.BytesIO(bytes(40 << 20))))
    pooled = {id(b) for b in C._POOL}
    assert pooled
    it = C.RabinChunkIter(_Ctx(), io.BytesIO(bytes(1 << 20)))
    next(it)
    assert id(it._segs[0][0]) in pooled or not it._segs


def test_read_error_after_earlier_reads(fake):
    """An error on a later read reaches the consumer after every chunk cut
    before it, then the iterator is finished (rabin.rs:131-138)."""
    from rustic_core_amd.errors import ErrorKind, RusticError
    data = bytes(40 << 20)

    class _Fail(io.RawIOBase):
        def __init__(self):
            self._b, self._calls = io.BytesIO(data), 0

        def readable(self):
            return True

        def readinto(self, mv):
            self._calls += 1
            if self._calls == 3:
                raise OSError("injected")
            b = self._b.read(len(mv))
            mv[:len(b)] = b
            return len(b)

    it = C.RabinChunkIter(_Ctx(), _Fail())
    got = []
    with pytest.raises(RusticError) as e:
        for c in it:
            got.append(len(c))
    assert e.value.kind == ErrorKind.InputOutput
    assert sum(got) <= 32 << 20 and it._stream.closed
    assert list(it) == []


@pytest.mark.parametrize("how", ["close", "del"])
def test_abandoned_iterator_waits_for_read_ahead(fake, monkeypatch, how):
    """A caller that stops early (close, or drops the iterator) while a read
    runs on the pipe's reader thread: the iterator waits for that read before its
    blocks can be freed or reused (the thread would otherwise
    write into a block another iterator owns)."""
    import threading
    import time
    monkeypatch.setenv("RCDC_READ_AHEAD", "1")
    log = []
    started = threading.Event()

    class _Slow(io.RawIOBase):
        def __init__(self):
            self.calls = 0

        def readable(self):
            return True

        def readinto(self, mv):
            self.calls += 1
            if self.calls >= 2:  # the pipe's reads (the first one's block is
                # fed before the consumer sees a cut: the next read runs)
                if self.calls >= 3:
                    started.set()
                time.sleep(0.3)
            mv[:len(mv)] = bytes(len(mv))
            log.append("read")
            return len(mv)

    it = C.RabinChunkIter(_Ctx(), _Slow())
    assert len(next(it)) == K
    assert started.wait(5) and it._pipe is not None
    blk = it._pipe.blk
    if how == "close":
        it.close()
    else:
        del it
        gc.collect()
    log.append("closed")
    assert log[-2:] == ["read", "closed"]
    assert blk.ptr or blk._keep is not None  # still a live block


def test_pipe_holds_at_most_pipe_blocks(fake):
    """A consumer that stops taking chunks: the pipe's reader stops once
    PIPE_BLOCKS blocks are read and not yet copied out, and resumes as the
    consumer retires blocks."""
    import time
    reads = []

    class _Count(io.RawIOBase):
        def __init__(self, n):
            self._b = io.BytesIO(bytes(n))

        def readable(self):
            return True

        def readinto(self, mv):
            reads.append(len(mv))
            b = self._b.read(len(mv))
            mv[:len(b)] = b
            return len(b)

    n = 200 << 20
    it = C.RabinChunkIter(_Ctx(), _Count(n))
    next(it)
    time.sleep(0.3)
    assert it._pipe is not None and len(reads) <= C.PIPE_BLOCKS
    total = K + sum(len(c) for c in it)
    assert total == n and len(reads) == n // C.READ_SIZE + 2  # (+ the last partial, EOF)


def test_pipe_never_waits_for_itself(monkeypatch):
    """The device stream hands out cuts only once it holds its pass size
    (16 MiB + 256) after its last cut, and a block goes back only when all
    of its bytes are copied out.  A last cut one byte before a block's end
    and reads short of 16 MiB then need a third block: with PIPE_BLOCKS = 2
    the round-6 pipe waited for itself (tools/soak_stream.py).  The bound is
    raised to what the stream needs (_pipe_blocks)."""
    import threading
    B = (16 << 20) + 256
    n = 64 << 20
    M = 1 << 20
    # cuts <= max (8 MiB) apart; the first pass (fed 31 MiB + 1) ends right
    # after the cut at 31 MiB, so its block keeps one unconsumed byte
    cuts_all = [8 * M, 16 * M, 24 * M, 31 * M, 38 * M, 46 * M, 54 * M, 62 * M, n]

    class _Batched:
        def __init__(self, ctx):
            self.fed, self.base, self.closed = 0, 0, False

        def feed(self, data, fin):
            self.fed += len(data)
            if not fin and self.fed - self.base < B:
                return np.zeros(0, np.uint64)
            out = [c for c in cuts_all if self.base < c < self.fed or (fin and c == self.fed)]
            if out:
                self.base = out[-1]
            return np.array(out, np.uint64)

        def close(self):
            self.closed = True

    class _Reads(io.RawIOBase):
        def __init__(self):
            self._b, self._first = io.BytesIO(bytes(n)), True

        def readable(self):
            return True

        def readinto(self, mv):
            k = len(mv) if self._first else min(len(mv), (15 << 20) + 1)
            self._first = False
            b = self._b.read(k)
            mv[:len(b)] = b
            return len(b)

    monkeypatch.setattr(C, "_Stream", _Batched)
    monkeypatch.setattr(C, "check_rabin_params", lambda *a: None)
    monkeypatch.setattr(C, "PIPE_BLOCKS", 2)
    got = []

    def run():
        got.extend(len(c) for c in C.RabinChunkIter(_Ctx(), _Reads()))
    t = threading.Thread(target=run, daemon=True)
    t.start()
    t.join(20)
    assert not t.is_alive(), "the pipe waited for itself"
    assert got == np.diff([0] + cuts_all).tolist()
