"""Minimal reader for R's RDX2/XDR serialization (the format of ``data/TD.rda``).

Test infrastructure only: used by ``make_td_fixture.py`` to turn the reference's
binary fixture ``/root/reference/data/TD.rda`` into plain ``.npz``/JSON golden
vectors.  Nothing here executes code from the file: it is a pure data decoder for
the subset of SEXP types that TD.rda contains (pairlists, generic vectors,
numeric/integer/logical/character vectors, symbols, language objects and
environments, with attributes).

Layout facts (R Internals, "Serialization Formats"): big-endian XDR, a flags word
per item with type in bits 0-7, object bit 8, attribute bit 9, tag bit 10.
"""
import bz2
import gzip
import struct

import numpy as np

NILVALUE, GLOBALENV, UNBOUNDVALUE, MISSINGARG, BASENAMESPACE = 254, 253, 252, 251, 250
NAMESPACESXP, PACKAGESXP, PERSISTSXP, REFSXP = 249, 248, 247, 255
EMPTYENV, BASEENV, ALTREP = 242, 241, 238
NA_INT = -2147483648


class RObj:
    """A decoded R object: ``value`` plus an ``attr`` dict (names, dim, class ...)."""

    def __init__(self, rtype, value, attr=None):
        self.rtype = rtype
        self.value = value
        self.attr = attr or {}

    def __repr__(self):
        return f"RObj(type={self.rtype}, attr={list(self.attr)})"

    # convenience accessors -------------------------------------------------
    def names(self):
        n = self.attr.get("names")
        return list(n.value) if n is not None else None

    def __getitem__(self, key):
        if isinstance(key, str):
            nm = self.names()
            return self.value[nm.index(key)]
        return self.value[key]

    def array(self):
        """Numeric vector → numpy, reshaped column-major by the ``dim`` attribute."""
        a = np.asarray(self.value)
        d = self.attr.get("dim")
        if d is not None:
            dims = tuple(int(x) for x in d.value)
            a = a.reshape(dims, order="F")
        return a


class _Reader:
    def __init__(self, buf):
        self.b = buf
        self.p = 0
        self.refs = []

    def i32(self):
        v = struct.unpack_from(">i", self.b, self.p)[0]
        self.p += 4
        return v

    def length(self):
        n = self.i32()
        if n == -1:
            hi, lo = self.i32(), self.i32()
            n = (hi << 32) + lo
        return n

    def item(self):
        flags = self.i32()
        t = flags & 0xFF
        has_attr = bool(flags & (1 << 9))
        has_tag = bool(flags & (1 << 10))
        if t == NILVALUE:
            return None
        if t in (EMPTYENV, BASEENV, GLOBALENV, UNBOUNDVALUE, MISSINGARG, BASENAMESPACE):
            return RObj(t, None)
        if t == REFSXP:
            idx = flags >> 8
            if idx == 0:
                idx = self.i32()
            return self.refs[idx - 1]
        if t in (NAMESPACESXP, PACKAGESXP, PERSISTSXP):
            self.i32()  # 0
            n = self.i32()
            strs = [self.item() for _ in range(n)]
            o = RObj(t, strs)
            self.refs.append(o)
            return o
        if t == 1:  # SYMSXP
            o = RObj(1, None)
            self.refs.append(o)
            o.value = self.item().value
            return o
        if t in (2, 3, 5, 6, 17):  # LISTSXP, CLOSXP, PROMSXP, LANGSXP, DOTSXP
            attr = self.item() if has_attr else None
            tag = self.item() if has_tag else None
            car = self.item()
            cdr = self.item()
            cell = RObj(t, (tag, car, cdr))
            if attr is not None:
                cell.attr = _pairlist_to_dict(attr)
            return cell
        if t == 4:  # ENVSXP
            locked = self.i32()
            o = RObj(4, None)
            self.refs.append(o)
            enclos = self.item()
            frame = self.item()
            hashtab = self.item()
            attr = self.item()
            o.value = dict(locked=locked, enclos=enclos, frame=frame, hashtab=hashtab)
            if attr is not None:
                o.attr = _pairlist_to_dict(attr)
            return o
        if t == 9:  # CHARSXP
            n = self.i32()
            if n == -1:
                return RObj(9, None)
            s = self.b[self.p:self.p + n].decode("utf-8", errors="replace")
            self.p += n
            return RObj(9, s)
        if t in (10, 13):  # LGLSXP, INTSXP
            n = self.length()
            a = np.frombuffer(self.b, dtype=">i4", count=n, offset=self.p).astype(np.int64)
            self.p += 4 * n
            o = RObj(t, a)
        elif t == 14:  # REALSXP
            n = self.length()
            a = np.frombuffer(self.b, dtype=">f8", count=n, offset=self.p).astype(np.float64)
            self.p += 8 * n
            o = RObj(t, a)
        elif t == 15:  # CPLXSXP
            n = self.length()
            a = np.frombuffer(self.b, dtype=">f8", count=2 * n, offset=self.p).astype(np.float64)
            self.p += 16 * n
            o = RObj(t, a[0::2] + 1j * a[1::2])
        elif t == 16:  # STRSXP
            n = self.length()
            o = RObj(16, [self.item().value for _ in range(n)])
        elif t in (19, 20):  # VECSXP, EXPRSXP
            n = self.length()
            o = RObj(t, [self.item() for _ in range(n)])
        elif t == 24:  # RAWSXP
            n = self.length()
            o = RObj(24, self.b[self.p:self.p + n])
            self.p += n
        elif t == 25:  # S4SXP
            o = RObj(25, None)
        else:
            raise ValueError(f"unsupported SEXP type {t} at offset {self.p}")
        if has_attr:
            o.attr = _pairlist_to_dict(self.item())
        return o


def _pairlist_to_dict(pl):
    out = {}
    while pl is not None and pl.rtype == 2:
        tag, car, cdr = pl.value
        out[tag.value if tag is not None else None] = car
        pl = cdr
    return out


def pairlist_items(pl):
    out = []
    while pl is not None and pl.rtype in (2, 6):
        tag, car, cdr = pl.value
        out.append((tag.value if tag is not None else None, car))
        pl = cdr
    return out


def read_rda(path):
    """Return ``{name: RObj}`` for every object saved in an .rda file."""
    raw = open(path, "rb").read()
    if raw[:3] == b"BZh":
        raw = bz2.decompress(raw)
    elif raw[:2] == b"\x1f\x8b":
        raw = gzip.decompress(raw)
    if not raw.startswith(b"RDX2\nX\n"):
        raise ValueError("not an RDX2/XDR file")
    r = _Reader(raw[7:])
    version = r.i32()
    r.i32()  # writer R version
    r.i32()  # min reader version
    if version == 3:
        n = r.i32()
        r.p += n  # native encoding string
    top = r.item()
    return dict(pairlist_items(top))
