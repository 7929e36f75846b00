"""Config 4's segment gather (BASELINE config 4): the .jpg bytes of a
batch whose frames are dealt over ranks (frame i on rank i mod N) are gathered to
rank 0, one message per rank.

Each rank packs its frames' bytes back to back with one kernel launch and moves
that run to rank 0 in ONE transfer.  Rank 0's batch buffer has a fixed region per rank
(rank r's run starts at r x cap_bytes), so no rank needs another rank's sizes to know
where its bytes go.  Two transports:
  - "p2p": RCCL over xGMI with the "nccl" backend (gloo with CPU tensors in the CPU
    tests): the run is one isend, matched by an irecv of exactly its size on rank 0;
  - "ipc": ranks that share one GPU (the --allow-shared-gpu rehearsal; RCCL refuses two
    ranks on one device): rank 0's batch buffers are opened in every rank through HIP
    IPC handles, and a rank's cat writes its run straight into its region of them.
The pack is one jpge_concat_segments launch (a HIP kernel, any byte alignment) on the
caller's current stream; CPU tensors (the gloo tests) use torch.cat.  The frame
lengths go to rank 0 alone, on a host-side gloo group (a few hundred bytes,
posted without waiting): rank 0 needs them to size its receives and to find frames.
No rank waits for another within a batch: rank 0 completes a batch's length receives
(and posts its p2p data receives) at the next post, so it starts its next encode
while the slowest rank is still finishing this one.

`post()` returns once the transfers are queued (nothing on the host waits for the GPU):
the next batch's encode runs while they move.  The caller encodes into two sets of
output slots alternately; `acquire()` names the set to encode into next, after the cat
that read it two batches earlier has finished (long since, in practice).  Two pack
and batch buffers alternate the same way.  Replaces nothing in the reference (a
single-process encoder); the bytes are the reference's files, unchanged.
"""
from __future__ import annotations

import ctypes
import time


class BatchGather:
    def __init__(self, group, meta_group, rank: int, world: int, nframes: int, cap_bytes: int, device,
                 transport: str = "p2p"):
        """group: the data-path group (RCCL, or gloo with CPU tensors; unused by "ipc");
        meta_group: a gloo group for the lengths; nframes: the batch; cap_bytes: the
        largest packed run one rank can send (its frames' capacities summed); device:
        where the pack and batch buffers live; transport: "p2p" or "ipc" (ranks on one
        GPU; falls back to "p2p" if the IPC handles cannot be opened)."""
        import torch
        import torch.distributed as dist

        self.dist, self.torch = dist, torch
        self.group, self.meta = group, meta_group
        self.rank, self.world, self.n = rank, world, nframes
        self.cap = cap_bytes
        self.nmax = (nframes + world - 1) // world
        self.cuda = torch.device(device).type == "cuda"
        self.pending = [[], []]   # works posted from each buffer (sends, receives, length messages)
        self.cat_ev = [None, None]  # the cat that read each output-slot set
        self.turn = 0
        self.last = 0
        self.got = [None, None]    # rank 0: every rank's lengths of the batch in buffer b
        self.where = [None, None]  # rank 0: frame offsets in batch[b] (built on first use)
        self._ptrs = {}            # the segments' device pointers (tuple) -> the same as a ctypes array (<= 4 kept)
        self.dev_index = torch.device(device).index if self.cuda else None
        if self.cuda and self.dev_index is None:
            self.dev_index = torch.cuda.current_device()
        self.lens_wait_s = 0.0     # rank 0: host time spent waiting for the other ranks' lengths
        self.lens_recv = [[], []]  # rank 0: the posted length receives of the batch in each buffer
        self.lens_out = [torch.zeros(self.nmax, dtype=torch.int64) for _ in range(2)]
        self.lens_all = [[torch.zeros(self.nmax, dtype=torch.int64) for _ in range(world)] for _ in range(2)]
        # rank 0: the batch, rank r's run at r * cap_bytes
        self.batch = [torch.empty(cap_bytes * world if rank == 0 else 1, dtype=torch.uint8, device=device)
                      for _ in range(2)]
        self.transport = "p2p"
        self.remote = None
        if transport == "ipc" and self.cuda and world > 1:
            self.remote = self._open_ipc()
            if self.remote is not None:
                self.transport = "ipc"
        # p2p senders pack into a buffer of their own (rank 0 packs into its region directly)
        self.packed = [torch.empty(cap_bytes if (rank and self.transport == "p2p") else 1, dtype=torch.uint8,
                                   device=device) for _ in range(2)]
        # every GPU operation of the gather (the concat launch, its events, the RCCL calls'
        # stream waits) runs on a stream of its own, never the null stream: an operation
        # there makes every later launch on the encoder's lane streams slower (the 4K
        # pipeline lost 3.5% to one memset)
        self.side = torch.cuda.Stream(device=self.dev_index) if self.cuda else None

    def _on_side(self):
        import contextlib

        return self.torch.cuda.stream(self.side) if self.side is not None else contextlib.nullcontext()

    def _open_ipc(self):
        """Every rank opens rank 0's two batch buffers (HIP IPC).  The handles travel over
        the gloo group; all ranks agree on the outcome, so either all use "ipc" or none."""
        torch, dist = self.torch, self.dist
        from torch.multiprocessing.reductions import reduce_tensor

        handles = [[reduce_tensor(t)[1] for t in self.batch] if self.rank == 0 else None]
        dist.broadcast_object_list(handles, src=dist.get_global_rank(self.meta, 0), group=self.meta)
        views, ok = None, 1
        if self.rank == 0:
            views = self.batch
        else:
            try:
                from torch.multiprocessing.reductions import rebuild_cuda_tensor

                views = [rebuild_cuda_tensor(*h) for h in handles[0]]
            except Exception:  # (an IPC-less runtime: fall back to p2p)
                ok = 0
        flag = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.meta)
        return views if int(flag) == 1 else None

    def share(self, r: int) -> list[int]:
        return list(range(r, self.n, self.world))

    def acquire(self) -> int:
        """The output-slot set (0/1) the caller encodes the next batch into."""
        ev = self.cat_ev[self.turn]
        if ev is not None:
            ev.synchronize()
            self.cat_ev[self.turn] = None
        return self.turn

    def post(self, segments, lens) -> None:
        """segments: this rank's frames' byte tensors (length >= lens[k] each), in share
        order, from the set acquire() named; lens: their .jpg lengths (host ints)."""
        with self._on_side():
            self._post(segments, lens)

    def _post(self, segments, lens) -> None:
        torch, dist = self.torch, self.dist
        b = self.turn
        self.turn ^= 1
        for w in self.pending[b]:  # (posted from these buffers two batches ago)
            w.wait()
        self.pending[b] = []
        lens = [int(n) for n in lens]
        total = sum(lens)
        if total > self.cap:
            raise ValueError(f"gather: {total} bytes exceed the rank's region of {self.cap}")
        meta0 = dist.get_global_rank(self.meta, 0)
        if self.rank:
            mine = self.lens_out[b]
            mine.zero_()
            if lens:
                mine[:len(lens)] = torch.tensor(lens, dtype=torch.int64)
            self.pending[b].append(dist.isend(mine, meta0, group=self.meta))
        # the run: rank 0 and "ipc" senders cat straight into their region of the batch
        if self.rank == 0:
            run = self.batch[b][:total]
        elif self.transport == "ipc":
            run = self.remote[b][self.rank * self.cap:self.rank * self.cap + total]
        else:
            run = self.packed[b][:total]
        if total and self.cuda:
            from . import concat_segments

            # (keyed by the pointers themselves, not the list object: a list reused with a
            # tensor replaced must not hand the kernel stale pointers; bounded, so
            # fresh lists per post do not pin old segments)
            key = tuple(t.data_ptr() for t in segments)
            arr = self._ptrs.get(key)
            if arr is None:
                if len(self._ptrs) >= 4:
                    self._ptrs.pop(next(iter(self._ptrs)))
                arr = self._ptrs[key] = (ctypes.c_void_p * len(key))(*key)
            concat_segments(self.dev_index, torch.cuda.current_stream().cuda_stream, arr,
                            (ctypes.c_size_t * len(lens))(*lens), run.data_ptr())
        elif total:
            torch.cat([seg[:n] for seg, n in zip(segments, lens) if n], out=run)
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record()
            self.cat_ev[b] = ev
        self.last = b
        if self.rank == 0:
            # this batch's lengths: receives posted now, completed at the next post (or
            # wait()), so rank 0 starts its next encode without waiting for the slowest
            # rank to finish this one; the previous batch's are completed first
            self._complete(b ^ 1)
            got = self.lens_all[b]
            got[0].zero_()
            if lens:
                got[0][:len(lens)] = torch.tensor(lens, dtype=torch.int64)
            self.lens_recv[b] = [dist.irecv(got[r], dist.get_global_rank(self.meta, r), group=self.meta)
                                 for r in range(1, self.world)]
            self.got[b] = got
            self.where[b] = None
        elif total and self.transport == "p2p":
            self.pending[b] += dist.batch_isend_irecv(
                [dist.P2POp(dist.isend, run, dist.get_global_rank(self.group, 0), group=self.group)])

    def _complete(self, b: int) -> None:
        """Rank 0: the length receives of the batch in buffer b, then (p2p) the receives of
        its runs, each exactly its size at its region."""
        waits = self.lens_recv[b]
        if not waits:
            return
        self.lens_recv[b] = []
        t0 = time.perf_counter()
        for w in waits:
            w.wait()
        self.lens_wait_s += time.perf_counter() - t0
        if self.transport != "p2p":
            return
        dist = self.dist
        ops = []
        for r in range(1, self.world):
            tot = int(self.got[b][r].sum())
            if tot:
                ops.append(dist.P2POp(dist.irecv, self.batch[b][r * self.cap:r * self.cap + tot],
                                      dist.get_global_rank(self.group, r), group=self.group))
        if ops:
            self.pending[b] += dist.batch_isend_irecv(ops)

    def wait(self) -> None:
        """Every posted transfer complete (rank 0: `batch` holds the last batch once every
        rank has returned from wait(), e.g. after a barrier)."""
        with self._on_side():
            self._wait()

    def _wait(self) -> None:
        for b in (self.last ^ 1, self.last):  # (the older batch's receives first, as they were posted)
            if self.rank == 0:
                self._complete(b)
        for b in (0, 1):
            for w in self.pending[b]:
                w.wait()
            self.pending[b] = []
            if self.cat_ev[b] is not None:
                self.cat_ev[b].synchronize()
        if self.cuda:
            self.torch.cuda.current_stream().synchronize()

    def frame(self, i: int):
        """Rank 0, after wait() on every rank: frame i's .jpg bytes in the latest batch (a view)."""
        b = self.last
        if self.where[b] is None:  # (frame i = share(i mod world)[i div world])
            self.where[b] = [[0] + [int(x) for x in self.got[b][r].cumsum(0)] for r in range(self.world)]
        r, k = i % self.world, i // self.world
        off = r * self.cap + self.where[b][r][k]
        return self.batch[b][off:off + self.where[b][r][k + 1] - self.where[b][r][k]]
