"""Host transport for rank mode without RCCL (jg_ctx_create_rank_transport): every exchange step of
the sharded engine staged through host memory and moved by torch.distributed (gloo, CPU).

For tests and rehearsals of the multi-process code paths on one GPU, where RCCL refuses two ranks on
one device; production rank mode uses RCCL (Context(unique_id=...)).
"""


class GlooTransport:
    """allgather / exchange of the jg_transport contract (include/janusgpu.h) over a torch.distributed
    process group (gloo, CPU tensors)."""

    def __init__(self, dist, world, group=None):
        self.dist, self.world, self.group = dist, world, group

    def allgather(self, data):
        import torch
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8) if data else torch.empty(0, dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t, group=self.group)
        return b"".join(o.numpy().tobytes() for o in out)

    def exchange(self, sends, recvs):
        import torch
        reqs, outs = [], []
        for peer, b in sends:
            reqs.append(self.dist.isend(torch.frombuffer(bytearray(b), dtype=torch.uint8), peer, group=self.group))
        for peer, nbytes in recvs:
            t = torch.empty(nbytes, dtype=torch.uint8)
            reqs.append(self.dist.irecv(t, peer, group=self.group))
            outs.append(t)
        for r in reqs:
            r.wait()
        return [t.numpy().tobytes() for t in outs]
