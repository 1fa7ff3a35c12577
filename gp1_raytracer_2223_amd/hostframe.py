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
import tempfile

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

    @staticmethod
    def _dirs() -> list[str]:
        return [SHM_DIR, tempfile.gettempdir()]

    @classmethod
    def create(cls, tag: str, nbytes: int) -> "SharedFrame":
        """In /dev/shm when it has room for the frame (a small container /dev/shm would raise
        SIGBUS on first touch of a page beyond it), else in the temp directory."""
        for d in cls._dirs():
            try:
                st = os.statvfs(d)
            except OSError:
                continue
            if st.f_bavail * st.f_frsize >= nbytes + (64 << 20):
                return cls(os.path.join(d, f"rtx_frame_{tag}"), nbytes, True)
        raise OSError(f"no room for a {nbytes}-byte shared frame in {cls._dirs()}")

    @classmethod
    def attach(cls, tag: str, nbytes: int) -> "SharedFrame":
        for d in cls._dirs():
            path = os.path.join(d, f"rtx_frame_{tag}")
            if os.path.exists(path):
                return cls(path, nbytes, False)
        raise FileNotFoundError(f"shared frame rtx_frame_{tag} not found in {cls._dirs()}")

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
