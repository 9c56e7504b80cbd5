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
import torch


def shard_first_frame(rank, batch, step=0, world=1):
    return step * world * batch + rank * batch


class BoundaryExchange:
    """Packs one frame's outputs (kcap x 28 B keypoints, kcap x 32 B
    descriptors, int32 count) into one buffer and all-gathers it."""

    def __init__(self, kcap, world, device):
        self.kcap, self.world = kcap, world
        self.nbytes = kcap * 60 + 16
        self.mine = torch.zeros(self.nbytes, dtype=torch.uint8, device=device)
        self.gathered = torch.zeros((world, self.nbytes), dtype=torch.uint8, device=device)

    def pack(self, kps, desc, count):
        k = self.kcap
        self.mine[:k * 28].copy_(kps.reshape(-1))
        self.mine[k * 28:k * 60].copy_(desc.reshape(-1))
        self.mine[k * 60:k * 60 + 4].copy_(count.reshape(1).view(torch.uint8))

    def exchange(self, dist, group=None):
        dist.all_gather_into_tensor(self.gathered.view(-1), self.mine, group=group)

    def ring_step(self, dist, rank, last, slot0, group=None):
        """After this step's extraction: last = (kps, desc, count) of this
        rank's last frame, slot0 = buffers receiving its first frame's
        predecessor (see module doc)."""
        if not hasattr(self, "carry"):
            self.carry = torch.zeros_like(self.mine)  # job-wide last frame of the previous step
        self.pack(*last)
        self.exchange(dist, group)
        if rank > 0:
            self.unpack_into(rank - 1, *slot0)
        else:
            self._unpack(self.carry, *slot0)
        self.carry.copy_(self.gathered[self.world - 1])

    def _unpack(self, src, kps, desc, count):
        k = self.kcap
        kps.copy_(src[:k * 28].view(k, 28))
        desc.copy_(src[k * 28:k * 60].view(k, 32))
        count.copy_(src[k * 60:k * 60 + 4].view(torch.int32).reshape(count.shape))

    def unpack_into(self, src_rank, kps, desc, count):
        k = self.kcap
        src = self.gathered[src_rank]
        kps.copy_(src[:k * 28].view(k, 28))
        desc.copy_(src[k * 28:k * 60].view(k, 32))
        count.copy_(src[k * 60:k * 60 + 4].view(torch.int32).reshape(count.shape))
