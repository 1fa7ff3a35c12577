"""Reader for the RTXB container written by oracle/ref/ref_harness (test infrastructure)."""
import struct

import numpy as np

_DT = {0: np.float32, 1: np.int32, 2: np.uint32, 3: np.uint8}


def read(path) -> dict:
    b = open(path, "rb").read()
    assert b[:4] == b"RTXB", path
    o, d = 4, {}
    while o < len(b):
        (nl,) = struct.unpack_from("<I", b, o)
        o += 4
        name = b[o:o + nl].decode()
        o += nl
        t, sz = struct.unpack_from("<IQ", b, o)
        o += 12
        d[name] = np.frombuffer(b[o:o + sz], dtype=_DT[t]).copy()
        o += sz
    return d
