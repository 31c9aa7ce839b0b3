"""Cross-shard transports of a sharded run for tgsim_set_transport.

With a transport attached, tgsim_advance / tgsim_advance_to_barrier run the window's exchange
themselves, a storm round MAX-reduces its batch's first / last time, and a signal batch is
all-gathered: a sharded run is driven with exactly the calls of a single-shard one, every call
collective over the shards. Multi-GPU runs use the library's native RCCL communicator
(tgsim_comm_init, Simulator.comm_init); the transports here are the caller-supplied form of the
same three operations:

  * GlooTransport - one process per shard over torch.distributed (gloo): the CPU tests (the oracle's
    host buffers) and bench.py's rehearsal of N ranks on fewer GPUs (device buffers staged through
    host memory);
  * ThreadGroup - several shards in one process, one thread each (tests on one GPU): peer blocks
    move by hipMemcpyAsync on the calling context's stream, or memmove for host buffers.

Operations follow include/tgsim.h: alltoall moves block p of every rank's send buffer to block
<rank> of rank p's receive buffer; allreduce_max_i64 is an element-wise MAX in place; allgather
concatenates every rank's bytes in rank order. An operation is complete when the callback returns.
"""
from __future__ import annotations

import ctypes as C
import threading
import traceback

import numpy as np

from . import _abi as A

_H2D, _D2H, _D2D = 1, 2, 3


def _hip():
    lib = C.CDLL("libamdhip64.so")
    lib.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
    lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    lib.hipStreamSynchronize.argtypes = [C.c_void_p]
    return lib


def _host(addr: int, nbytes: int) -> np.ndarray:
    return np.frombuffer((C.c_uint8 * nbytes).from_address(addr), dtype=np.uint8) if nbytes else np.zeros(0, np.uint8)


class Transport:
    """The C struct of callbacks (kept alive with this object). Subclasses implement alltoall,
    allreduce_max and allgather on raw addresses; a raised exception becomes the error code -1."""

    def __init__(self):
        def wrap(f):
            def cb(_user, *args):
                try:
                    f(*args)
                    return 0
                except Exception:  # the library turns -1 into TGSIM_EHIP with a message
                    traceback.print_exc()
                    return -1
            return cb
        def abort_cb(_user):
            try:
                self.abort()
            except Exception:  # noqa: BLE001 - an abort must not raise into the library
                traceback.print_exc()
        self._cbs = (A.ALLTOALL_FN(wrap(self.alltoall)), A.ALLREDUCE_FN(wrap(self.allreduce_max)),
                     A.ALLGATHER_FN(wrap(self.allgather)), A.ABORT_FN(abort_cb))
        self.c = A.Transport(None, *self._cbs)

    def abort(self):
        """tgsim_transport.abort: this shard failed; the peers' pending and later collectives must
        fail instead of waiting for it."""

    def alltoall(self, send, recv, block, stream):
        raise NotImplementedError

    def allreduce_max(self, buf, n, stream):
        raise NotImplementedError

    def allgather(self, send, recv, nbytes, stream):
        raise NotImplementedError


class GlooTransport(Transport):
    """One shard per process over torch.distributed (gloo, host tensors). device=True: the library's
    buffers are device memory (HIP contexts), staged through host copies after a stream sync."""

    def __init__(self, dist, device: bool = False):
        super().__init__()
        self.dist, self.device = dist, device
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.hip = _hip() if device else None

    def _get(self, addr, nbytes, stream):
        if not self.device:
            return _host(addr, nbytes)
        out = np.empty(nbytes, np.uint8)
        assert self.hip.hipStreamSynchronize(stream) == 0
        if nbytes:
            assert self.hip.hipMemcpy(out.ctypes.data, addr, nbytes, _D2H) == 0
        return out

    def _put(self, addr, arr):
        if not self.device:
            if len(arr):
                _host(addr, len(arr))[:] = arr
            return
        if len(arr):
            assert self.hip.hipMemcpy(addr, arr.ctypes.data, len(arr), _H2D) == 0

    def abort(self):
        # the peers' gloo collectives fail once this rank's connections close
        self.dist.destroy_process_group()

    def alltoall(self, send, recv, block, stream):
        import torch
        s = torch.from_numpy(self._get(send, block * self.world, stream).copy())
        r = torch.empty_like(s)
        self.dist.all_to_all_single(r, s)
        mine = r.numpy()
        if self.device:
            self._put(recv, mine)
        else:  # the own block stays untouched (k_recv / tgo_advance_end skip it)
            dst = _host(recv, block * self.world)
            for p in range(self.world):
                if p != self.rank:
                    dst[p * block:(p + 1) * block] = mine[p * block:(p + 1) * block]

    def allreduce_max(self, buf, n, stream):
        import torch
        t = torch.from_numpy(self._get(buf, 8 * n, stream).view(np.int64).copy())
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        self._put(buf, t.numpy().view(np.uint8))

    def allgather(self, send, recv, nbytes, stream):
        import torch
        s = torch.from_numpy(self._get(send, nbytes, stream).copy())
        parts = [torch.empty_like(s) for _ in range(self.world)]
        self.dist.all_gather(parts, s)
        out = torch.cat(parts).numpy()
        self._put(recv, out)


class ThreadGroup:
    """n shards of one process, each driven by its own thread; member(k) is shard k's transport.
    device=True: HIP contexts on one device (blocks move by hipMemcpyAsync on the caller's stream)."""

    def __init__(self, n: int, device: bool = False, timeout: float = 300.0):
        self.n, self.device = n, device
        self.bar = threading.Barrier(n, timeout=timeout)
        self.slot = [None] * n
        self.hip = _hip() if device else None

    def member(self, k: int) -> Transport:
        return _ThreadMember(self, k)


class _ThreadMember(Transport):
    def __init__(self, g: ThreadGroup, k: int):
        super().__init__()
        self.g, self.k = g, k

    def abort(self):
        self.g.bar.abort()   # every pending and later wait raises BrokenBarrierError -> -1

    def _sync(self, stream):
        if self.g.device:
            assert self.g.hip.hipStreamSynchronize(stream) == 0

    def _copy(self, dst, src, nbytes, stream):
        if not nbytes:
            return
        if self.g.device:
            assert self.g.hip.hipMemcpyAsync(dst, src, nbytes, _D2D, stream) == 0
        else:
            C.memmove(dst, src, nbytes)

    def alltoall(self, send, recv, block, stream):
        g, k = self.g, self.k
        self._sync(stream)            # this shard's send blocks are complete
        g.slot[k] = send
        g.bar.wait()
        for p in range(g.n):
            if p != k:
                self._copy(recv + p * block, g.slot[p] + k * block, block, stream)
        self._sync(stream)            # the copies are done before any peer moves on
        g.bar.wait()

    def _host_values(self, addr, nbytes, stream):
        if not self.g.device:
            return _host(addr, nbytes).copy()
        out = np.empty(nbytes, np.uint8)
        self._sync(stream)
        if nbytes:
            assert self.g.hip.hipMemcpy(out.ctypes.data, addr, nbytes, _D2H) == 0
        return out

    def _write(self, addr, arr):
        if not len(arr):
            return
        if self.g.device:
            assert self.g.hip.hipMemcpy(addr, arr.ctypes.data, len(arr), _H2D) == 0
        else:
            _host(addr, len(arr))[:] = arr

    def allreduce_max(self, buf, n, stream):
        g, k = self.g, self.k
        g.slot[k] = self._host_values(buf, 8 * n, stream).view(np.int64)
        g.bar.wait()
        m = np.max(np.stack(g.slot), axis=0)
        g.bar.wait()
        self._write(buf, m.astype(np.int64).view(np.uint8))

    def allgather(self, send, recv, nbytes, stream):
        g, k = self.g, self.k
        g.slot[k] = self._host_values(send, nbytes, stream)
        g.bar.wait()
        out = np.concatenate(g.slot)
        g.bar.wait()
        self._write(recv, out)


def run_threads(fns):
    """Run fns[k]() on one thread each; returns their results in order (re-raises the first error)."""
    res, err = [None] * len(fns), [None] * len(fns)

    def go(k):
        try:
            res[k] = fns[k]()
        except BaseException as e:  # noqa: BLE001 - handed to the caller
            err[k] = e

    ts = [threading.Thread(target=go, args=(k,)) for k in range(len(fns))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in err:
        if e is not None:
            raise e
    return res
