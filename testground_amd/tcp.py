"""TCP-level view of a simulation.

``tgsim_tcp_send`` segments application writes into packets that take the per-packet path;
``tgsim_tcp_react`` (after every window) recovers lost or corrupted segments by retransmission and
completes writes. This module adds what a receiving application sees on a connection: the byte
stream is in order, so write k of connection (src, dst) is readable at

    t_app[k] = max(t_app[k - 1], t_done[k])

in write order ((t_send, seq) on the connection); a write that is still pending holds back every
later one, and one that failed resets the connection, failing every later write at its time
(Go's ``net.Conn.Write`` / ``Read`` then return an error: ``plans/benchmarks/storm.go:163-168``).
"""
from __future__ import annotations

import numpy as np

from . import _abi as A

PENDING, DELIVERED, TIMEOUT, REFUSED = A.TCP_PENDING, A.TCP_DELIVERED, A.TCP_TIMEOUT, A.TCP_REFUSED
NEVER = np.iinfo(np.int64).max


def in_order(src, dst, seq, t_send, state, t_done):
    """Per write: (state, t_app) as the receiving application reads it, from the writes (in send
    order: src, dst, seq, t_send) and their transport outcome (state, t_done from tgsim_tcp_writes).
    Pending -> t_app = NEVER."""
    src, dst = np.asarray(src, np.int64), np.asarray(dst, np.int64)
    seq, t_send = np.asarray(seq, np.int64), np.asarray(t_send, np.int64)
    state, t_done = np.asarray(state, np.int64), np.asarray(t_done, np.int64)
    n = len(src)
    order = np.lexsort((np.arange(n), seq, t_send, dst, src))
    out_state = np.empty(n, np.int64)
    out_t = np.empty(n, np.int64)
    i = 0
    while i < n:
        j = i
        while j < n and src[order[j]] == src[order[i]] and dst[order[j]] == dst[order[i]]:
            j += 1
        run, blocked, t = order[i:j], None, np.iinfo(np.int64).min
        for w in run:
            if blocked is not None:
                out_state[w], out_t[w] = blocked
                continue
            s = state[w]
            if s == DELIVERED:
                t = max(t, int(t_done[w]))
                out_state[w], out_t[w] = DELIVERED, t
            elif s == PENDING:
                blocked = (PENDING, NEVER)
                out_state[w], out_t[w] = blocked
            else:
                blocked = (s, int(t_done[w]))
                out_state[w], out_t[w] = blocked
        i = j
    return out_state, out_t
