"""A host frame shared by the ranks' processes: the gather target of the multi-GPU path.

SURVEY §8(e): the frame's 16-row stripes are rendered on G GPUs and gathered on the host —
no collective, no peer traffic.  With one process per GPU (bench.py under torchrun) the
gather target is one page-locked mapping of a /dev/shm file that every rank maps; each
rank's `rtx_gather_async` writes only the rows it owns, straight from its GPU over its own
PCIe link.  The file is unlinked as soon as every rank has mapped it, so nothing is left
in /dev/shm even if a rank dies later.

    f = SharedFrame.create(tag, nbytes)   # rank 0, before the barrier
    f = SharedFrame.attach(tag, nbytes)   # other ranks, after it
    f.unlink()                            # rank 0, after a second barrier
    f.pin(ctx)                            # hipHostRegister through the C-ABI
"""
from __future__ import annotations

import ctypes as C
import mmap
import os

import numpy as np

from . import abi

SHM_DIR = "/dev/shm"


class SharedFrame:
    def __init__(self, path: str, nbytes: int, create: bool):
        self.path = path
        self.nbytes = int(nbytes)
        flags = os.O_RDWR | (os.O_CREAT | os.O_EXCL if create else 0)
        fd = os.open(path, flags, 0o600)
        try:
            if create:
                os.ftruncate(fd, self.nbytes)
            self.mm = mmap.mmap(fd, self.nbytes, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        finally:
            os.close(fd)
        self.buf = np.frombuffer(self.mm, dtype=np.uint8)
        self._pinned = None

    @classmethod
    def create(cls, tag: str, nbytes: int) -> "SharedFrame":
        return cls(os.path.join(SHM_DIR, f"rtx_frame_{tag}"), nbytes, True)

    @classmethod
    def attach(cls, tag: str, nbytes: int) -> "SharedFrame":
        return cls(os.path.join(SHM_DIR, f"rtx_frame_{tag}"), nbytes, False)

    def unlink(self) -> None:
        try:
            os.unlink(self.path)
        except FileNotFoundError:
            pass

    def view(self, dtype, count: int, offset: int = 0) -> np.ndarray:
        return np.frombuffer(self.mm, dtype=dtype, count=count, offset=offset)

    def address(self) -> int:
        return self.buf.ctypes.data

    def pin(self, ctx) -> bool:
        """Page-lock the mapping for DMA (hipHostRegister).  False if the runtime refused
        (the gather then goes through pageable staging: correct, slower)."""
        rc = ctx.lib.rtx_host_register(ctx.h, C.c_void_p(self.address()), self.nbytes)
        if rc == abi.RTX_OK:
            self._pinned = ctx
            return True
        return False

    def close(self) -> None:
        if self._pinned is not None and getattr(self._pinned, "h", None):
            self._pinned.lib.rtx_host_unregister(self._pinned.h, C.c_void_p(self.address()))
        self._pinned = None
        self.buf = None
        try:
            self.mm.close()
        except BufferError:   # a numpy view is still alive; the mapping goes with the process
            pass
