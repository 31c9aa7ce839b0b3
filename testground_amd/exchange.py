"""The per-window exchange step of a sharded run, as the runner drives it over
torch.distributed (RCCL on GPUs, gloo in the CPU tests).

A context's exchange buffer holds one block of `xcap` records per peer; record 0 of a block is a
header whose `t` field is the number of records that follow (written on the device by the window's
token bucket, include/tgsim.h). Only those records travel: the counts are exchanged first (one
small all-to-all), then the blocks' used prefixes in one variable-size all-to-all, and the received
prefixes are placed back at their block offsets for tgsim_advance_end. Moving the full fixed-size
buffers instead would cost S x xcap x 32 B per rank per window regardless of the traffic."""
from __future__ import annotations

REC = 32  # bytes per tgsim_record


def exchange(send, recv, xcap: int, dist) -> int:
    """All-to-all of the used part of every peer block. send / recv: uint8 tensors of
    world * xcap * 32 bytes (device tensors for RCCL, CPU tensors for gloo). Returns the number of
    records received from other ranks. One host round trip (the counts)."""
    import torch

    world, rank = dist.get_world_size(), dist.get_rank()
    blk = xcap * REC
    cnt = send.view(torch.int64).view(world, xcap * 4)[:, 0].contiguous()
    cnt_in = torch.empty_like(cnt)
    dist.all_to_all_single(cnt_in, cnt)
    both = torch.stack([cnt, cnt_in]).cpu().tolist()
    out_n = [(1 + min(max(int(c), 0), xcap - 1)) * REC for c in both[0]]
    in_n = [(1 + min(max(int(c), 0), xcap - 1)) * REC for c in both[1]]
    out_n[rank] = in_n[rank] = REC  # nothing to send to oneself but the header
    packed = torch.cat([send[p * blk:p * blk + out_n[p]] for p in range(world)])
    packed_in = torch.empty(sum(in_n), dtype=torch.uint8, device=send.device)
    dist.all_to_all_single(packed_in, packed, output_split_sizes=in_n, input_split_sizes=out_n)
    off = 0
    for p in range(world):
        if p != rank:
            recv[p * blk:p * blk + in_n[p]].copy_(packed_in[off:off + in_n[p]])
        off += in_n[p]
    return sum(in_n[p] // REC - 1 for p in range(world) if p != rank)
