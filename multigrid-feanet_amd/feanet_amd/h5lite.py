"""Read-only access to the reference's HDF5 datasets without h5py.

The reference's datasets (`Data/IsoPoisson/*.h5`, `Data/TestPoisson/*.h5`, `Data/RHS/*.h5`) are read by
`Data/dataset.py:11-13, 29-33, 56-57, 73-80` through `h5py.File(path)[name]`; h5py is not installed in
this image.  Those files use the original HDF5 format (superblock v0/v1, v1 object headers,
symbol-table groups) with contiguous or compact little/big-endian float/int datasets, which is all this
reader supports: anything else (chunked or filtered storage, v2+ superblocks, compound types) raises
`NotImplementedError` naming what it found, so a file it cannot read fails loudly instead of
returning wrong data.

Usage mirrors the slice of h5py the reference uses::

    with File(path) as h5:
        a = np.array(h5["rhs"], dtype=np.float32)   # h5["rhs"] is a numpy array (memory-mapped)
        names = list(h5.keys())
"""
import mmap

import numpy as np

_SIG = b"\x89HDF\r\n\x1a\n"
_UNDEF = 0xFFFFFFFFFFFFFFFF


class _Reader:
    def __init__(self, buf, so, sl):
        self.b, self.so, self.sl = buf, so, sl

    def u(self, pos, n):
        return int.from_bytes(self.b[pos:pos + n], "little")

    def off(self, pos):
        return self.u(pos, self.so)

    def ln(self, pos):
        return self.u(pos, self.sl)


class File:
    """Minimal `h5py.File(path, 'r')` stand-in: `keys()`, `[name]` (nested 'a/b' paths too), `close()`."""

    def __init__(self, path, mode="r"):
        if mode != "r":
            raise ValueError("h5lite.File is read-only")
        self._fh = open(path, "rb")
        self._mm = mmap.mmap(self._fh.fileno(), 0, access=mmap.ACCESS_READ)
        self.filename = path
        base = self._find_superblock()
        b = self._mm
        ver = b[base + 8]
        if ver not in (0, 1):
            raise NotImplementedError(f"{path}: HDF5 superblock version {ver} (only 0/1 supported)")
        so, sl = b[base + 13], b[base + 14]
        self._r = _Reader(b, so, sl)
        p = base + 24 + (4 if ver == 1 else 0)
        self._base = self._r.off(p)
        p += 4 * so  # base, free-space, end-of-file, driver-info addresses
        root_ohdr = self._r.off(p + so)  # root symbol-table entry: link-name offset, object header
        self._root = self._group_links(root_ohdr)

    # -- plumbing --------------------------------------------------------------------------
    def _find_superblock(self):
        pos = 0
        while pos + 8 <= len(self._mm):
            if self._mm[pos:pos + 8] == _SIG:
                return pos
            pos = 512 if pos == 0 else pos * 2
        raise ValueError(f"{self.filename}: not an HDF5 file")

    def _addr(self, a):
        return self._base + a

    def _messages(self, ohdr):
        """Yield (type, data_pos, size) of a v1 object header, following continuation blocks."""
        r, b = self._r, self._mm
        p = self._addr(ohdr)
        if b[p:p + 4] == b"OHDR":
            raise NotImplementedError(f"{self.filename}: v2 object headers are not supported")
        if b[p] != 1:
            raise NotImplementedError(f"{self.filename}: object header version {b[p]}")
        nmsg = r.u(p + 2, 2)
        blocks = [(p + 16, r.u(p + 8, 4))]
        seen = 0
        while blocks and seen < nmsg:
            q, size = blocks.pop(0)
            end = q + size
            while q + 8 <= end and seen < nmsg:
                mtype, msize = r.u(q, 2), r.u(q + 2, 2)
                seen += 1
                if mtype == 0x10:  # continuation: offset, length
                    blocks.append((self._addr(r.off(q + 8)), r.ln(q + 8 + r.so)))
                else:
                    yield mtype, q + 8, msize
                q += 8 + msize

    def _heap_name(self, heap, off):
        b, r = self._mm, self._r
        h = self._addr(heap)
        if b[h:h + 4] != b"HEAP":
            raise ValueError(f"{self.filename}: bad local heap")
        data = self._addr(r.off(h + 8 + 2 * r.sl))
        end = b.find(b"\0", data + off)
        return bytes(b[data + off:end]).decode()

    def _group_links(self, ohdr):
        """name -> object header address for a symbol-table (old-style) group; None for a dataset."""
        st = None
        for mtype, q, _ in self._messages(ohdr):
            if mtype == 0x11:
                st = (self._r.off(q), self._r.off(q + self._r.so))
            elif mtype in (0x02, 0x06, 0x0A):
                raise NotImplementedError(f"{self.filename}: new-style (link message) groups")
        if st is None:
            return None
        links = {}
        self._walk_btree(st[0], st[1], links)
        return links

    def _walk_btree(self, node, heap, links):
        b, r = self._mm, self._r
        p = self._addr(node)
        if b[p:p + 4] != b"TREE" or b[p + 4] != 0:
            raise ValueError(f"{self.filename}: bad group B-tree node")
        level, used = b[p + 5], r.u(p + 6, 2)
        q = p + 8 + 2 * r.so + r.sl  # first child (after key 0)
        for _ in range(used):
            child = r.off(q)
            if level > 0:
                self._walk_btree(child, heap, links)
            else:
                s = self._addr(child)
                if b[s:s + 4] != b"SNOD":
                    raise ValueError(f"{self.filename}: bad symbol table node")
                nsym = r.u(s + 6, 2)
                e = s + 8
                for _ in range(nsym):
                    links[self._heap_name(heap, r.off(e))] = r.off(e + r.so)
                    e += 2 * r.so + 24
            q += r.so + r.sl

    def _dataset(self, ohdr, name):
        b, r = self._mm, self._r
        shape = dtype = layout = None
        for mtype, q, _ in self._messages(ohdr):
            if mtype == 0x01:
                ver, nd = b[q], b[q + 1]
                d0 = q + (8 if ver == 1 else 4)
                shape = tuple(r.ln(d0 + i * r.sl) for i in range(nd))
            elif mtype == 0x03:
                dtype = self._dtype(q, name)
            elif mtype == 0x08:
                layout = self._layout(q, name)
            elif mtype == 0x0B:
                raise NotImplementedError(f"{self.filename}:{name}: filtered (compressed) storage")
        if shape is None or dtype is None or layout is None:
            raise NotImplementedError(f"{self.filename}:{name}: not a plain dataset")
        count = int(np.prod(shape, dtype=np.int64)) if shape else 1
        kind, where = layout
        if kind == "contiguous":
            if where == _UNDEF:  # never written: h5py reads the fill value (0)
                return np.zeros(shape, dtype)
            arr = np.frombuffer(self._mm, dtype=dtype, count=count, offset=self._addr(where))
        else:
            arr = np.frombuffer(bytes(where), dtype=dtype, count=count)
        return arr.reshape(shape)

    def _dtype(self, q, name):
        b, r = self._mm, self._r
        cls, bits0, size = b[q] & 0x0F, b[q + 1], r.u(q + 4, 4)
        endian = ">" if bits0 & 1 else "<"
        if cls == 1 and size in (2, 4, 8):
            return np.dtype(f"{endian}f{size}")
        if cls == 0 and size in (1, 2, 4, 8):
            return np.dtype(f"{endian}{'i' if bits0 & 8 else 'u'}{size}")
        raise NotImplementedError(f"{self.filename}:{name}: datatype class {cls} size {size}")

    def _layout(self, q, name):
        b, r = self._mm, self._r
        ver = b[q]
        if ver == 3:
            cls = b[q + 1]
            if cls == 1:
                return "contiguous", r.off(q + 2)
            if cls == 0:
                n = r.u(q + 2, 2)
                return "compact", b[q + 4:q + 4 + n]
        elif ver in (1, 2):
            nd, cls = b[q + 1], b[q + 2]
            if cls == 1:
                return "contiguous", r.off(q + 8)
            if cls == 0:
                p = q + 8 + 4 * nd
                n = r.u(p, 4)
                return "compact", b[p + 4:p + 4 + n]
        raise NotImplementedError(f"{self.filename}:{name}: layout version {ver} (chunked storage?)")

    # -- h5py-like surface ------------------------------------------------------------------
    def keys(self):
        return list(self._root or {})

    def __contains__(self, name):
        return name in (self._root or {})

    def __getitem__(self, name):
        links = self._root
        parts = [p for p in name.split("/") if p]
        for i, part in enumerate(parts):
            if links is None or part not in links:
                raise KeyError(f"{name!r} not in {self.filename}")
            ohdr = links[part]
            if i < len(parts) - 1:
                links = self._group_links(ohdr)
        if self._group_links(ohdr) is not None:
            raise NotImplementedError(f"{name!r} is a group; read its datasets by path")
        return self._dataset(ohdr, name)

    def close(self):
        # arrays returned by [] view the mapping; copy them (np.array(...)) before closing
        try:
            self._mm.close()
        except BufferError:
            pass  # views still alive: the mapping is released with them
        self._fh.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
