"""Config 4's segment gather (BASELINE config 4): the .jpg bytes of a
batch whose frames are dealt over ranks (frame i on rank i mod N) are gathered to
rank 0, one message per rank.

Each rank packs its frames' bytes back to back in a device buffer with one
`torch.cat` launch, and sends that run as ONE point-to-point message (RCCL over
xGMI with the "nccl" backend; gloo in the CPU tests).  The frame lengths travel
ahead on a host-side gloo group (a few hundred bytes, no device synchronisation), so
rank 0 posts its receives with exact sizes at exact places: rank r's run lands at
the sum of the lower ranks' runs, in the order of its frames.

`post()` returns as soon as the messages are queued: the next batch's encode runs
while they move (the encoder's lanes have streams of their own).  Two pack buffers
alternate; a buffer is reused only after the messages posted from it two batches
earlier have completed.  Replaces nothing in the reference (a single-process
encoder); the bytes are the reference's files, unchanged.
"""
from __future__ import annotations


class BatchGather:
    def __init__(self, group, meta_group, rank: int, world: int, nframes: int, cap_bytes: int, device):
        """group: the data-path group (RCCL, or gloo with CPU tensors); meta_group: a
        gloo group for the lengths; nframes: the batch; cap_bytes: the largest packed
        run one rank can send (its frames' capacities summed); device: where the pack
        buffers live (rank 0's receive buffer too)."""
        import torch
        import torch.distributed as dist

        self.dist, self.torch = dist, torch
        self.group, self.meta = group, meta_group
        self.rank, self.world, self.n = rank, world, nframes
        self.nmax = (nframes + world - 1) // world
        self.packed = [torch.empty(cap_bytes, dtype=torch.uint8, device=device) for _ in range(2)]
        self.pending = [[], []]  # work handles of the messages posted from each pack buffer
        self.turn = 0
        # rank 0: the whole batch, packed by rank (rank r's run after the runs of ranks < r),
        # one buffer per pack buffer (a batch's receives never overlap the previous one's)
        self.batch = [torch.empty(cap_bytes * world if rank == 0 else 1, dtype=torch.uint8, device=device)
                      for _ in range(2)]
        self.lens_all = [torch.zeros(self.nmax, dtype=torch.int64) for _ in range(world)]
        self.where = [None, None]  # rank 0: frame i -> (offset in batch[b], length)
        self.last = 0              # the buffer of the latest post

    def share(self, r: int) -> list[int]:
        return list(range(r, self.n, self.world))

    def post(self, segments, lens) -> None:
        """segments: this rank's frames' byte tensors (length >= lens[k] each), in
        share order; lens: their .jpg lengths (host ints)."""
        torch, dist = self.torch, self.dist
        b = self.turn
        self.turn ^= 1
        for w in self.pending[b]:  # (the messages sent from this buffer two batches ago)
            w.wait()
        self.pending[b] = []
        mine = torch.zeros(self.nmax, dtype=torch.int64)
        mine[:len(lens)] = torch.tensor(list(lens), dtype=torch.int64)
        dist.all_gather(self.lens_all, mine, group=self.meta)
        total = int(sum(lens))
        run = self.packed[b][:total]
        torch.cat([seg[:n] for seg, n in zip(segments, lens)], out=run)
        if run.is_cuda:  # the caller's next encode rewrites the segments: the pack must be done
            ev = torch.cuda.Event()
            ev.record()
            ev.synchronize()
        totals = [int(t.sum()) for t in self.lens_all]
        self.last = b
        if self.rank == 0:
            ops = []
            base = totals[0]
            dst = self.batch[b]
            dst[:total].copy_(run)
            for r in range(1, self.world):
                if totals[r]:
                    ops.append(dist.P2POp(dist.irecv, dst[base:base + totals[r]],
                                          dist.get_global_rank(self.group, r), group=self.group))
                base += totals[r]
            where = {}
            base = 0
            for r in range(self.world):
                off = base
                for k, i in enumerate(self.share(r)):
                    n = int(self.lens_all[r][k])
                    where[i] = (off, n)
                    off += n
                base += totals[r]
            self.where[b] = where
        else:
            ops = [dist.P2POp(dist.isend, run, dist.get_global_rank(self.group, 0), group=self.group)] if total else []
        if ops:
            self.pending[b] = dist.batch_isend_irecv(ops)

    def wait(self) -> None:
        """Every posted message complete (rank 0: `batch` holds the last batch)."""
        for b in (0, 1):
            for w in self.pending[b]:
                w.wait()
            self.pending[b] = []

    def frame(self, i: int):
        """Rank 0, after wait(): frame i's .jpg bytes in the latest batch (a view)."""
        off, n = self.where[self.last][i]
        return self.batch[self.last][off:off + n]
