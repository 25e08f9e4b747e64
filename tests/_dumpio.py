"""Reader for the SWDUMP1 record files written by oracle/refdump.c and by the
framework's own state export (test infrastructure only)."""
from __future__ import annotations

import numpy as np


def read_dump(path: str) -> dict:
    out: dict = {}
    with open(path, "rb") as f:
        buf = f.read()
    if buf[:7] != b"SWDUMP1":
        raise ValueError("not a SWDUMP1 file: %s" % path)
    pos = 8
    n = len(buf)
    while pos < n:
        name = buf[pos:pos + 48].split(b"\0", 1)[0].decode()
        dt = chr(buf[pos + 48])
        cnt = int(np.frombuffer(buf, dtype="<i8", count=1, offset=pos + 49)[0])
        pos += 57
        dtype = "<f8" if dt == "d" else "<i4"
        size = 8 if dt == "d" else 4
        out[name] = np.frombuffer(buf, dtype=dtype, count=cnt, offset=pos).copy()
        pos += cnt * size
    nn, nl = int(out["counts"][0]), int(out["counts"][1])
    for k, v in list(out.items()):
        if k.startswith("s.node."):
            out[k] = v.reshape(-1, nn)
        elif k.startswith("s.link."):
            out[k] = v.reshape(-1, nl)
    return out
