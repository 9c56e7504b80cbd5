"""Frame sharding and the one exchange step of the multi-GPU path.

Frames are sharded in contiguous blocks: rank r of W processes global frames
[step*W*B + r*B, step*W*B + (r+1)*B).  Extraction needs no communication;
matching frame t against t-1 crosses a rank boundary once per rank and step:
after extraction every rank all-gathers its last frame's (keypoints,
descriptors, count); rank r > 0 takes rank r-1's entry of this step, rank 0
takes rank W-1's entry of the previous step (the job's frame before its
first one), kept from the previous exchange.  With the "nccl" backend this
is an RCCL all-gather over xGMI; tests run it with gloo on CPU.
"""
import ctypes

import torch


def shard_first_frame(rank, batch, step=0, world=1):
    return step * world * batch + rank * batch


class BoundaryExchange:
    """Packs one frame's outputs (kcap x 28 B keypoints, kcap x 32 B
    descriptors, int32 count) into one buffer and all-gathers it."""

    def __init__(self, kcap, world, device):
        self.kcap, self.world = kcap, world
        self.nbytes = kcap * 60 + 16  # = orbx_boundary_record_bytes(kcap)
        self.mine = torch.zeros(self.nbytes, dtype=torch.uint8, device=device)
        # two all-gather targets used alternately: rank 0 reads the previous
        # step's last record from the other one (no carry copy)
        self._bufs = [torch.zeros((world, self.nbytes), dtype=torch.uint8, device=device)
                      for _ in range(2)]
        self._step = 0
        self.gathered = self._bufs[0]

    def _native(self, kps, desc, count, src=None):
        # device-resident exchange (RCCL): one liborbx launch per pack /
        # unpack (orbx_boundary_pack / _unpack) instead of three tensor copies.
        # The launch trusts its pointers, so every size and the device are
        # checked here; anything else takes the (checked) tensor copies.
        ts = (kps, desc, count) + ((src,) if src is not None else ())
        if not (self.mine.is_cuda and all(t.is_cuda and t.is_contiguous() for t in ts)):
            return False
        cur = torch.cuda.current_device()
        k = self.kcap
        return (all(t.device.index == cur for t in ts + (self.mine,))
                and kps.numel() * kps.element_size() >= k * 28
                and desc.numel() * desc.element_size() >= k * 32
                and count.numel() * count.element_size() >= 4
                and (src is None or src.numel() * src.element_size() >= self.nbytes))

    def pack(self, kps, desc, count):
        k = self.kcap
        if self._native(kps, desc, count):
            import orbx
            orbx._check(orbx.lib().orbx_boundary_pack(
                ctypes.c_void_p(kps.data_ptr()), ctypes.c_void_p(desc.data_ptr()),
                ctypes.c_void_p(count.data_ptr()), k, ctypes.c_void_p(self.mine.data_ptr()),
                orbx._stream_handle(None)), "orbx_boundary_pack")
            return
        self.mine[:k * 28].copy_(kps.reshape(-1))
        self.mine[k * 28:k * 60].copy_(desc.reshape(-1))
        self.mine[k * 60:k * 60 + 4].copy_(count.reshape(1).view(torch.uint8))

    def exchange(self, dist, group=None):
        dist.all_gather_into_tensor(self.gathered.view(-1), self.mine, group=group)

    def ring_step(self, dist, rank, last, slot0, group=None):
        """After this step's extraction: last = (kps, desc, count) of this
        rank's last frame, slot0 = buffers receiving its first frame's
        predecessor (see module doc)."""
        prev = self.gathered  # previous step's records (zeros before the first step)
        self.gathered = self._bufs[self._step & 1]
        if self._step == 0:
            prev = self._bufs[1]
        self._step += 1
        self.pack(*last)
        self.exchange(dist, group)
        if rank > 0:
            self.unpack_into(rank - 1, *slot0)
        else:  # the job-wide last frame of the previous step
            self._unpack(prev[self.world - 1], *slot0)

    def _unpack(self, src, kps, desc, count):
        k = self.kcap
        if self._native(kps, desc, count, src):
            import orbx
            orbx._check(orbx.lib().orbx_boundary_unpack(
                ctypes.c_void_p(src.data_ptr()), k, ctypes.c_void_p(kps.data_ptr()),
                ctypes.c_void_p(desc.data_ptr()), ctypes.c_void_p(count.data_ptr()),
                orbx._stream_handle(None)), "orbx_boundary_unpack")
            return
        kps.copy_(src[:k * 28].view(k, 28))
        desc.copy_(src[k * 28:k * 60].view(k, 32))
        count.copy_(src[k * 60:k * 60 + 4].view(torch.int32).reshape(count.shape))

    def unpack_into(self, src_rank, kps, desc, count):
        self._unpack(self.gathered[src_rank], kps, desc, count)
