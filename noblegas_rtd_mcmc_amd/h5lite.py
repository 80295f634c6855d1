"""A small HDF5 reader and writer for netCDF-4 files: the container of the reference's traces.

The reference saves every run with ``az.to_netcdf`` (age_ens_runs_mcmc/run_age_mcmc_utils.py
:420-425, ng_interp/noble_gas_mcmc.py:422-447): one netCDF-4 file, i.e. an HDF5 file with
the netCDF-4 conventions (dimension scales, ``_Netcdf4Dimid``, ``_NCProperties``), and reads
it back with ``az.from_netcdf`` (run_age_mcmc_utils.py:434, run_age_mcmc.post_plots.comp.py
:171, age_modeling_mcmc.post_plots.py:128).  h5py / netCDF4 / xarray are not in this image,
so this module implements the part of the HDF5 file format (format specification 3.0) those
files use, from the specification, in plain Python (struct + zlib):

Reader (``H5Reader``): superblock v0-v3; object headers v1 and v2 with continuation
blocks; compact and dense (fractal heap + v2 B-tree) link and attribute storage; symbol-table
(v1 B-tree + local heap) groups; datatypes fixed-point, floating-point, string, compound,
reference and variable-length; dataspaces v1/v2; compact, contiguous and chunked (v1 B-tree)
layouts with the deflate / shuffle / fletcher32 filters; global heap collections (variable-
length data: the DIMENSION_LIST attributes).

Writer (``H5Writer``, ``write_netcdf4``): superblock v2 and version-2 object headers
(lookup3 checksums) with compact link and attribute storage; datasets as one chunk with the
shuffle + deflate filters behind a one-entry v1 B-tree (the layout the shipped traces use) or
contiguous; fixed-length string, numeric, variable-length object-reference and compound
attributes; one global heap collection.  That is what a netCDF-4 reader needs from the file:
groups, variables, the dimension scales with their REFERENCE_LIST back-references, every
variable's DIMENSION_LIST and netCDF's _Netcdf4Dimid / _Netcdf4Coordinates / _NCProperties.
"""
import struct
import os
import zlib

import numpy as np

UNDEF = 0xFFFFFFFFFFFFFFFF
_SIG = b"\x89HDF\r\n\x1a\n"
_M32 = 0xFFFFFFFF


# ------------------------------------------------------------------ checksum
def _rot(x, k):
    return ((x << k) | (x >> (32 - k))) & _M32


def lookup3(data, initval=0):
    """Bob Jenkins' lookup3 hashlittle() over bytes, as HDF5's H5_checksum_lookup3 (the
    checksum of every version-2 metadata structure)."""
    n = len(data)
    a = b = c = (0xDEADBEEF + n + initval) & _M32
    i = 0
    while n > 12:
        a = (a + int.from_bytes(data[i:i + 4], "little")) & _M32
        b = (b + int.from_bytes(data[i + 4:i + 8], "little")) & _M32
        c = (c + int.from_bytes(data[i + 8:i + 12], "little")) & _M32
        a = (a - c) & _M32; a ^= _rot(c, 4); c = (c + b) & _M32
        b = (b - a) & _M32; b ^= _rot(a, 6); a = (a + c) & _M32
        c = (c - b) & _M32; c ^= _rot(b, 8); b = (b + a) & _M32
        a = (a - c) & _M32; a ^= _rot(c, 16); c = (c + b) & _M32
        b = (b - a) & _M32; b ^= _rot(a, 19); a = (a + c) & _M32
        c = (c - b) & _M32; c ^= _rot(b, 4); b = (b + a) & _M32
        n -= 12
        i += 12
    if n == 0:
        return c
    tail = bytes(data[i:i + n]) + b"\0" * (12 - n)
    a = (a + int.from_bytes(tail[0:4], "little")) & _M32
    b = (b + int.from_bytes(tail[4:8], "little")) & _M32
    c = (c + int.from_bytes(tail[8:12], "little")) & _M32
    c ^= b; c = (c - _rot(b, 14)) & _M32
    a ^= c; a = (a - _rot(c, 11)) & _M32
    b ^= a; b = (b - _rot(a, 25)) & _M32
    c ^= b; c = (c - _rot(b, 16)) & _M32
    a ^= c; a = (a - _rot(c, 4)) & _M32
    b ^= a; b = (b - _rot(a, 14)) & _M32
    c ^= b; c = (c - _rot(b, 24)) & _M32
    return c


class H5Error(ValueError):
    pass


# ------------------------------------------------------------------ datatypes
class Dtype:
    """A parsed datatype message: cls (0 fixed, 1 float, 3 string, 6 compound, 7 reference,
    9 vlen), size, and per class: signed / order, pad / charset, members, base, vkind."""

    def __init__(self, cls, size, **kw):
        self.cls, self.size = cls, size
        self.__dict__.update(kw)

    def numpy(self):
        if self.cls == 0:
            return np.dtype(("<" if self.order == 0 else ">") + ("i" if self.signed else "u") + str(self.size))
        if self.cls == 1:
            return np.dtype(("<" if self.order == 0 else ">") + "f" + str(self.size))
        if self.cls == 3:
            return np.dtype("S%d" % self.size)
        if self.cls == 7:
            return np.dtype("<u8")
        if self.cls == 6:
            return np.dtype({"names": [m[0] for m in self.members], "formats": [m[2].numpy() for m in self.members],
                             "offsets": [m[1] for m in self.members], "itemsize": self.size})
        raise H5Error("no numpy dtype for class %d" % self.cls)

    def describe(self):
        """A comparable description (structure diffs)."""
        if self.cls == 0:
            return "int%d%s" % (8 * self.size, "" if self.signed else "u")
        if self.cls == 1:
            return "float%d" % (8 * self.size)
        if self.cls == 3:
            return "string%d" % self.size
        if self.cls == 7:
            return "objref"
        if self.cls == 9:
            return "vlen(%s)" % ("string" if self.vkind == 1 else self.base.describe())
        if self.cls == 6:
            return "compound(%s)" % ",".join("%s:%s" % (m[0], m[2].describe()) for m in self.members)
        return "class%d" % self.cls


def parse_dtype(b, o=0):
    """Datatype message at b[o:] -> (Dtype, bytes consumed)."""
    cv = b[o]
    cls, ver = cv & 0x0F, cv >> 4
    bits = b[o + 1] | (b[o + 2] << 8) | (b[o + 3] << 16)
    size = struct.unpack_from("<I", b, o + 4)[0]
    p = o + 8
    if cls == 0:
        return Dtype(0, size, order=bits & 1, signed=bool(bits & 8)), 12
    if cls == 1:
        return Dtype(1, size, order=bits & 1), 20
    if cls == 2:
        return Dtype(2, size), 8 + 2 + 2
    if cls == 3:
        return Dtype(3, size, pad=bits & 0x0F, charset=(bits >> 4) & 0x0F), 8
    if cls == 7:
        return Dtype(7, size, rtype=bits & 0x0F), 8
    if cls == 9:
        base, n = parse_dtype(b, p)
        return Dtype(9, size, vkind=bits & 0x03, pad=(bits >> 2) & 0x03, charset=(bits >> 8) & 0x0F, base=base), 8 + n
    if cls == 6:
        nmem = bits & 0xFFFF
        members = []
        for _ in range(nmem):
            e = b.index(b"\0", p)
            name = bytes(b[p:e]).decode()
            if ver < 3:
                p += ((e - p) // 8 + 1) * 8
                off = struct.unpack_from("<I", b, p)[0]
                p += 4
                if ver == 1:
                    p += 1 + 3 + 4 + 4 + 16     # dimensionality, reserved, perm, reserved, dims
            else:
                p = e + 1
                nb = max(1, (size.bit_length() + 7) // 8)
                off = int.from_bytes(b[p:p + nb], "little")
                p += nb
            mt, n = parse_dtype(b, p)
            p += n
            members.append((name, off, mt))
        return Dtype(6, size, members=members), p - o
    if cls == 10:       # array
        rank = b[p]
        p += 1 if ver >= 3 else 4
        dims = struct.unpack_from("<%dI" % rank, b, p)
        p += 4 * rank
        if ver < 3:
            p += 4 * rank
        base, n = parse_dtype(b, p)
        return Dtype(10, size, dims=dims, base=base), p + n - o
    raise H5Error("unsupported datatype class %d" % cls)


def parse_dataspace(b, o, L):
    ver, rank, flags = b[o], b[o + 1], b[o + 2]
    if ver == 1:
        p = o + 8
        kind = 1 if rank else 0
    else:
        kind = b[o + 3]
        p = o + 4
    dims = tuple(int.from_bytes(b[p + L * i:p + L * (i + 1)], "little") for i in range(rank))
    if kind == 2:
        return None                       # null dataspace
    return dims


# ------------------------------------------------------------------ reader
class H5Reader:
    """Read-only view of an HDF5 file (bytes).  ``tree()`` returns the nested
    {group: {"attrs", "groups", "datasets"}} structure; datasets as numpy arrays."""

    def __init__(self, path_or_bytes):
        if isinstance(path_or_bytes, (bytes, bytearray, memoryview)):
            self.b = bytes(path_or_bytes)
        else:
            with open(path_or_bytes, "rb") as f:
                self.b = f.read()
        b = self.b
        base = 0
        while b[base:base + 8] != _SIG:
            base = 512 if base == 0 else base * 2
            if base >= len(b):
                raise H5Error("not an HDF5 file")
        self.sb_ver = b[base + 8]
        if self.sb_ver in (2, 3):
            self.O, self.L = b[base + 9], b[base + 10]
            p = base + 12
            self.base = self._addr(p); p += self.O
            p += self.O                                   # superblock extension
            self.eof = self._addr(p); p += self.O
            self.root = self._addr(p); p += self.O
            if lookup3(b[base:p]) != struct.unpack_from("<I", b, p)[0]:
                raise H5Error("superblock checksum mismatch")
        elif self.sb_ver in (0, 1):
            self.O, self.L = b[base + 13], b[base + 14]
            p = base + 16 + 4 + (4 if self.sb_ver == 1 else 0)
            self.base = self._addr(p); p += self.O
            p += self.O                                   # free-space info
            self.eof = self._addr(p); p += self.O
            p += self.O                                   # driver info
            # root group symbol table entry: link name offset, object header address, ...
            self.root = self._addr(p + self.O)
        else:
            raise H5Error("superblock version %d" % self.sb_ver)
        self._gheap = {}

    def _addr(self, p):
        return int.from_bytes(self.b[p:p + self.O], "little")

    def _len(self, p):
        return int.from_bytes(self.b[p:p + self.L], "little")

    # -------------------------------------------------------------- object headers
    def messages(self, addr):
        """[(type, flags, bytes)] of the object header at addr (continuations followed)."""
        b = self.b
        out = []
        if b[addr:addr + 4] == b"OHDR":
            flags = b[addr + 5]
            p = addr + 6
            if flags & 0x20:
                p += 16
            if flags & 0x10:
                p += 4
            nsz = 1 << (flags & 3)
            size0 = int.from_bytes(b[p:p + nsz], "little")
            p += nsz
            chunks = [(p, p + size0, flags)]
            if lookup3(b[addr:p + size0]) != struct.unpack_from("<I", b, p + size0)[0]:
                raise H5Error("object header checksum mismatch at %d" % addr)
            ci = 0
            while ci < len(chunks):
                s, e, fl = chunks[ci]
                q = s
                while q + 4 <= e:
                    mt, ms, mf = b[q], struct.unpack_from("<H", b, q + 1)[0], b[q + 3]
                    q += 4 + (2 if fl & 0x04 else 0)
                    data = b[q:q + ms]
                    q += ms
                    if mt == 0x10:                       # continuation
                        ca, cl = self._addr_of(data, 0), int.from_bytes(data[self.O:self.O + self.L], "little")
                        if b[ca:ca + 4] != b"OCHK":
                            raise H5Error("bad continuation block")
                        chunks.append((ca + 4, ca + cl - 4, fl))
                    else:
                        out.append((mt, mf, data))
                ci += 1
            return out
        if b[addr] == 1:                                  # version-1 object header
            nmsg = struct.unpack_from("<H", b, addr + 2)[0]
            size0 = struct.unpack_from("<I", b, addr + 8)[0]
            chunks = [(addr + 16, addr + 16 + size0)]
            ci = 0
            while ci < len(chunks) and len(out) < nmsg:
                s, e = chunks[ci]
                q = s
                while q + 8 <= e:
                    mt, ms, mf = struct.unpack_from("<HHB", b, q)
                    data = b[q + 8:q + 8 + ms]
                    q += 8 + ms
                    if mt == 0x10:
                        ca, cl = self._addr_of(data, 0), int.from_bytes(data[self.O:self.O + self.L], "little")
                        chunks.append((ca, ca + cl))
                    else:
                        out.append((mt, mf, data))
                ci += 1
            return out
        raise H5Error("no object header at %d" % addr)

    def _addr_of(self, data, p):
        return int.from_bytes(data[p:p + self.O], "little")

    # -------------------------------------------------------------- fractal heap + v2 B-tree
    def _fheap(self, addr):
        b = self.b
        if b[addr:addr + 4] != b"FRHP":
            raise H5Error("no fractal heap at %d" % addr)
        p = addr + 5
        h = {}
        h["id_len"], h["filt_len"] = struct.unpack_from("<HH", b, p); p += 4
        h["flags"] = b[p]; p += 1
        p += 4                                            # max managed object size
        p += self.L + self.O + self.L + self.O + 4 * self.L + 4 * self.L
        h["width"] = struct.unpack_from("<H", b, p)[0]; p += 2
        h["start"] = self._len(p); p += self.L
        h["max_direct"] = self._len(p); p += self.L
        h["max_heap_bits"] = struct.unpack_from("<H", b, p)[0]; p += 2
        p += 2                                            # starting rows in root indirect block
        h["root"] = self._addr(p); p += self.O
        h["rows"] = struct.unpack_from("<H", b, p)[0]; p += 2
        h["off_bytes"] = (h["max_heap_bits"] + 7) // 8
        return h

    def _fheap_obj(self, h, hid):
        """Managed (or tiny) object of the heap h for heap ID bytes hid."""
        kind = (hid[0] >> 4) & 3
        if kind == 2:                                    # tiny: the data is in the ID
            n = (hid[0] & 0x0F) + 1
            return hid[1:1 + n]
        if kind != 0:
            raise H5Error("huge fractal-heap objects are not supported")
        ob = h["off_bytes"]
        off = int.from_bytes(hid[1:1 + ob], "little")
        ln = int.from_bytes(hid[1 + ob:h["id_len"]], "little")
        blk, boff = self._fheap_block(h, off)
        return self.b[blk + boff:blk + boff + ln]

    def _fheap_block(self, h, off):
        """(direct block address, offset of `off` inside that block)."""
        if h["rows"] == 0:
            return h["root"], off
        # root indirect block: rows of `width` direct blocks, sizes start, start, 2 start, ...
        b = self.b
        ib = h["root"]
        p = ib + 5 + self.O + h["off_bytes"]
        pos, row, col = 0, 0, 0
        while True:
            size = h["start"] * (1 if row < 2 else 1 << (row - 1))
            if size > h["max_direct"]:
                raise H5Error("indirect fractal-heap rows are not supported")
            addr = self._addr(p)
            p += self.O + (self.L + 4 if h["filt_len"] else 0)
            if pos <= off < pos + size:
                return addr, off - pos
            pos += size
            col += 1
            if col == h["width"]:
                col, row = 0, row + 1

    def _btree2_records(self, addr):
        b = self.b
        if b[addr:addr + 4] != b"BTHD":
            raise H5Error("no v2 B-tree at %d" % addr)
        rsize = struct.unpack_from("<H", b, addr + 10)[0]
        depth = struct.unpack_from("<H", b, addr + 12)[0]
        root = self._addr(addr + 16)
        nroot = struct.unpack_from("<H", b, addr + 16 + self.O)[0]
        total = self._len(addr + 18 + self.O)
        nsize = struct.unpack_from("<I", b, addr + 6)[0]
        out = []

        def node(a, n, d):
            p = a + 6
            recs = [b[p + i * rsize:p + (i + 1) * rsize] for i in range(n)]
            if d == 0:
                out.extend(recs)
                return
            p += n * rsize
            # child pointers: address, records in child (bytes to encode the max records of
            # a node), [total records below if d > 1]
            maxrec = (nsize - 10) // rsize
            cb = max(1, (maxrec.bit_length() + 7) // 8)
            tb = max(1, (total.bit_length() + 7) // 8)
            for i in range(n + 1):
                ca = self._addr(p); p += self.O
                cn = int.from_bytes(b[p:p + cb], "little"); p += cb
                if d > 1:
                    p += tb
                node(ca, cn, d - 1)
                if i < n:
                    out.append(recs[i])
        if root != UNDEF and nroot:
            node(root, nroot, depth)
        return out

    # -------------------------------------------------------------- links
    def links(self, addr):
        """{name: object header address} of the group at addr."""
        msgs = self.messages(addr)
        out = {}
        dense = None
        for mt, _, d in msgs:
            if mt == 0x06:
                name, target = self._link(d)
                if target is not None:
                    out[name] = target
            elif mt == 0x02:
                fl = d[1]
                p = 2 + (8 if fl & 1 else 0)
                fh, bt = self._addr_of(d, p), self._addr_of(d, p + self.O)
                if fh != UNDEF:
                    dense = (fh, bt)
            elif mt == 0x11:                              # symbol table (old-style group)
                out.update(self._symtab(self._addr_of(d, 0), self._addr_of(d, self.O)))
        if dense:
            h = self._fheap(dense[0])
            for rec in self._btree2_records(dense[1]):
                name, target = self._link(self._fheap_obj(h, rec[4:]))
                if target is not None:
                    out[name] = target
        return out

    def _link(self, d):
        fl = d[1]
        p = 2
        ltype = 0
        if fl & 0x08:
            ltype = d[p]; p += 1
        if fl & 0x04:
            p += 8
        if fl & 0x10:
            p += 1
        nb = 1 << (fl & 3)
        nlen = int.from_bytes(d[p:p + nb], "little"); p += nb
        name = bytes(d[p:p + nlen]).decode(); p += nlen
        return name, (self._addr_of(d, p) if ltype == 0 else None)

    def _symtab(self, btree, lheap):
        b = self.b
        data_addr = self._addr(lheap + 8 + 2 * self.L)
        out = {}

        def walk(a):
            if b[a:a + 4] != b"TREE":
                raise H5Error("bad group B-tree")
            level, n = b[a + 5], struct.unpack_from("<H", b, a + 6)[0]
            p = a + 8 + 2 * self.O + self.L
            for _ in range(n):
                child = self._addr(p); p += self.O + self.L
                if level:
                    walk(child)
                else:
                    if b[child:child + 4] != b"SNOD":
                        raise H5Error("bad symbol node")
                    cnt = struct.unpack_from("<H", b, child + 6)[0]
                    q = child + 8
                    for _ in range(cnt):
                        no = self._len(q)
                        oh = self._addr(q + self.O)
                        e = b.index(b"\0", data_addr + no)
                        out[b[data_addr + no:e].decode()] = oh
                        q += 2 * self.O + 4 + 4 + 16
        walk(btree)
        return out

    # -------------------------------------------------------------- attributes
    def attrs(self, addr, raw=False):
        """{name: value} of the object at addr (raw: (Dtype, dims, value))."""
        out = {}
        for mt, _, d in self.messages(addr):
            if mt == 0x0C:
                name, v = self._attr(d)
                out[name] = v
            elif mt == 0x15:
                fl = d[1]
                p = 2 + (2 if fl & 1 else 0)
                fh, bt = self._addr_of(d, p), self._addr_of(d, p + self.O)
                if fh != UNDEF:
                    h = self._fheap(fh)
                    for rec in self._btree2_records(bt):
                        name, v = self._attr(self._fheap_obj(h, rec[:8]))
                        out[name] = v
        if raw:
            return out
        return {k: v[2] for k, v in out.items()}

    def _attr(self, d):
        ver = d[0]
        if ver == 1:
            nlen, tlen, slen = struct.unpack_from("<HHH", d, 2)
            p = 8
            name = bytes(d[p:p + nlen]).rstrip(b"\0").decode(); p += (nlen + 7) // 8 * 8
            dt, _ = parse_dtype(d, p); p += (tlen + 7) // 8 * 8
            dims = parse_dataspace(d, p, self.L); p += (slen + 7) // 8 * 8
        else:
            nlen, tlen, slen = struct.unpack_from("<HHH", d, 2)
            p = 8 if ver == 2 else 9
            name = bytes(d[p:p + nlen]).rstrip(b"\0").decode(); p += nlen
            dt, _ = parse_dtype(d, p); p += tlen
            dims = parse_dataspace(d, p, self.L); p += slen
        return name, (dt, dims, self._value(dt, dims, d[p:]))

    def _value(self, dt, dims, raw):
        if dims is None:
            return None
        n = int(np.prod(dims)) if dims else 1
        if dt.cls == 9:
            vals = []
            for i in range(n):
                p = i * (4 + self.O + 4)
                cnt = struct.unpack_from("<I", raw, p)[0]
                col = self._addr_of(raw, p + 4)
                idx = struct.unpack_from("<I", raw, p + 4 + self.O)[0]
                blob = self._gheap_obj(col, idx) if cnt else b""
                if dt.vkind == 1:
                    vals.append(blob.decode())
                else:
                    vals.append(np.frombuffer(blob, dtype=dt.base.numpy(), count=cnt))
            return vals if dims else vals[0]
        arr = np.frombuffer(bytes(raw[:n * dt.size]), dtype=dt.numpy(), count=n)
        if dt.cls == 3:
            s = [x.split(b"\0")[0].decode() for x in arr]
            return s[0] if not dims else s
        if not dims:
            return arr[0]
        return arr.reshape(dims)

    def _gheap_obj(self, col, idx):
        if col not in self._gheap:
            b = self.b
            if b[col:col + 4] != b"GCOL":
                raise H5Error("no global heap at %d" % col)
            size = self._len(col + 8)
            objs = {}
            p = col + 8 + self.L
            while p + 8 + self.L <= col + size:
                i = struct.unpack_from("<H", b, p)[0]
                sz = self._len(p + 8)
                if i == 0:
                    break
                objs[i] = b[p + 8 + self.L:p + 8 + self.L + sz]
                p += 8 + self.L + (sz + 7) // 8 * 8
            self._gheap[col] = objs
        return self._gheap[col][idx]

    # -------------------------------------------------------------- datasets
    def is_dataset(self, addr):
        return any(mt == 0x08 for mt, _, _ in self.messages(addr))

    def dataset_info(self, addr):
        dt = dims = layout = None
        filters = []
        for mt, _, d in self.messages(addr):
            if mt == 0x01:
                dims = parse_dataspace(d, 0, self.L)
            elif mt == 0x03:
                dt, _ = parse_dtype(d, 0)
            elif mt == 0x08:
                layout = d
            elif mt == 0x0B:
                filters = self._filters(d)
        return dt, dims, layout, filters

    def _filters(self, d):
        ver, n = d[0], d[1]
        p = 8 if ver == 1 else 2
        out = []
        for _ in range(n):
            fid = struct.unpack_from("<H", d, p)[0]; p += 2
            nlen = 0
            if ver == 1 or fid >= 256:
                nlen = struct.unpack_from("<H", d, p)[0]; p += 2
            flags, ncd = struct.unpack_from("<HH", d, p); p += 4
            if ver == 1:
                p += (nlen + 7) // 8 * 8
            else:
                p += nlen
            cd = struct.unpack_from("<%dI" % ncd, d, p); p += 4 * ncd
            if ver == 1 and ncd % 2:
                p += 4
            out.append((fid, cd))
        return out

    def read(self, addr):
        """The dataset at addr as a numpy array."""
        dt, dims, lay, filters = self.dataset_info(addr)
        if dims is None:
            return None
        n = int(np.prod(dims)) if dims else 1
        ver, cls = lay[0], lay[1]
        if ver < 3:
            raise H5Error("layout message version %d" % ver)
        if cls == 0:
            sz = struct.unpack_from("<H", lay, 2)[0]
            raw = lay[4:4 + sz]
        elif cls == 1:
            a = self._addr_of(lay, 2)
            raw = b"" if a == UNDEF else self.b[a:a + n * dt.size]
        elif cls == 2 and ver == 3:
            rank = lay[2] - 1
            bt = self._addr_of(lay, 3)
            cdims = struct.unpack_from("<%dI" % (rank + 1), lay, 3 + self.O)[:rank]
            raw = self._chunks(bt, dims, cdims, dt.size, filters)
        else:
            raise H5Error("layout class %d (version %d)" % (cls, ver))
        if dt.cls == 9 or dt.cls == 3:
            return self._value(dt, dims, raw)
        if len(raw) < n * dt.size:            # never written: the fill value (0 here)
            raw = bytes(raw) + b"\0" * (n * dt.size - len(raw))
        return np.frombuffer(bytes(raw[:n * dt.size]), dtype=dt.numpy(), count=n).reshape(dims).copy()

    def _chunks(self, bt, dims, cdims, esize, filters):
        out = np.zeros(int(np.prod(dims)) * esize, dtype=np.uint8).reshape(tuple(dims) + (esize,))
        if bt == UNDEF:
            return out.tobytes()
        b = self.b
        rank = len(dims)

        def walk(a):
            if b[a:a + 4] != b"TREE" or b[a + 4] != 1:
                raise H5Error("bad chunk B-tree")
            level, n = b[a + 5], struct.unpack_from("<H", b, a + 6)[0]
            p = a + 8 + 2 * self.O
            ksz = 8 + 8 * (rank + 1)
            for _ in range(n):
                csize, fmask = struct.unpack_from("<II", b, p)
                offs = struct.unpack_from("<%dQ" % rank, b, p + 8)
                child = self._addr(p + ksz)
                p += ksz + self.O
                if level:
                    walk(child)
                    continue
                data = b[child:child + csize]
                for i, (fid, cd) in reversed(list(enumerate(filters))):
                    if fmask & (1 << i):
                        continue
                    if fid == 1:
                        data = zlib.decompress(data)
                    elif fid == 2:
                        es = cd[0] if cd else esize
                        m = len(data) // es
                        data = np.frombuffer(data, np.uint8)[:m * es].reshape(es, m).T.tobytes() + data[m * es:]
                    elif fid == 3:
                        data = data[:-4]
                    else:
                        raise H5Error("filter %d" % fid)
                blk = np.frombuffer(data, np.uint8)[:int(np.prod(cdims)) * esize].reshape(tuple(cdims) + (esize,))
                sl = tuple(slice(o, min(o + c, d)) for o, c, d in zip(offs, cdims, dims))
                out[sl] = blk[tuple(slice(0, s.stop - s.start) for s in sl)]
        walk(bt)
        return out.tobytes()

    # -------------------------------------------------------------- whole tree
    def tree(self, addr=None, data=True):
        """{"attrs": {...}, "groups": {name: subtree}, "datasets": {name: {"attrs", "dtype",
        "shape", "data"}}} of the group at addr (default: the root)."""
        addr = self.root if addr is None else addr
        node = {"attrs": self.attrs(addr), "groups": {}, "datasets": {}, "addr": addr}
        for name, a in self.links(addr).items():
            if self.is_dataset(a):
                dt, dims, _, filters = self.dataset_info(a)
                node["datasets"][name] = {"attrs": self.attrs(a), "dtype": dt, "shape": dims, "addr": a,
                                          "filters": [f[0] for f in filters],
                                          "data": self.read(a) if data else None}
            else:
                node["groups"][name] = self.tree(a, data)
        return node


# ------------------------------------------------------------------ writer
def _dtype_msg(kind, size=8, signed=True, base=None, members=None):
    """Datatype message bytes: kind 'int' | 'float' | 'string' (fixed length, NULLTERM,
    ASCII) | 'objref' | 'vlen' (sequence of base) | 'compound' (members (name, offset, msg))."""
    if kind == "int":
        return struct.pack("<BBBBI", 0x10, 0x08 if signed else 0, 0, 0, size) + struct.pack("<HH", 0, 8 * size)
    if kind == "float":
        if size == 8:
            return struct.pack("<BBBBI", 0x11, 0x20, 0x3F, 0, 8) + struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
        return struct.pack("<BBBBI", 0x11, 0x20, 0x1F, 0, 4) + struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
    if kind == "string":
        return struct.pack("<BBBBI", 0x13, 0, 0, 0, size)
    if kind == "objref":
        return struct.pack("<BBBBI", 0x17, 0, 0, 0, 8)
    if kind == "vlen":
        return struct.pack("<BBBBI", 0x19, 0, 0, 0, 16) + base
    if kind == "compound":               # version 1: names padded to 8 bytes, 4-byte offsets
        body = b""
        for name, off, mt in members:
            nb = name.encode() + b"\0"
            body += nb + b"\0" * (-len(nb) % 8) + struct.pack("<I", off) + b"\0" * 28 + mt
        return struct.pack("<BBBBI", 0x16, len(members) & 0xFF, len(members) >> 8, 0, size) + body
    raise ValueError(kind)


def _dataspace_msg(dims, maxdims=False):
    """Dataspace message v2: scalar (dims None) or simple (maxdims = dims when asked)."""
    if dims is None:
        return struct.pack("<BBBB", 2, 0, 0, 0)
    d = b"".join(struct.pack("<Q", int(x)) for x in dims)
    return struct.pack("<BBBB", 2, len(dims), 1 if maxdims else 0, 1) + d + (d if maxdims else b"")


_CHUNK_K = 32                                     # v1 B-tree K of chunked datasets (the default)
# chunk byte bound: netCDF-4's default chunk size (NC_DEFAULT_CHUNK_SIZE, 4 MiB).  A variable
# up to it is ONE chunk (the shipped traces' 3 x 10 000 draws are), a larger one is tiled.
CHUNK_BYTES = 4 << 20


def chunk_dims(shape, itemsize, limit=None):
    """Chunk shape of a variable: the whole shape while it fits in ``limit`` bytes, else the
    largest axis halved (rounded up) until it fits; zero-length axes get chunk extent 1
    (HDF5 requires positive chunk dimensions; such a variable stores no chunk at all)."""
    limit = CHUNK_BYTES if limit is None else limit
    cd = [max(1, int(d)) for d in shape]
    while int(np.prod(cd)) * itemsize > limit:
        i = int(np.argmax(cd))
        if cd[i] == 1:
            break
        cd[i] = (cd[i] + 1) // 2
    return tuple(cd)


class H5Writer:
    """Builds an HDF5 file: superblock v2, version-2 object headers (lookup3 checksums),
    compact link and attribute storage, numeric datasets either contiguous or chunked with
    the shuffle + deflate filters (chunk_dims: one chunk up to 4 MiB, else tiled; a v1 B-tree
    chunk index of as many levels as the chunk count needs, 2K = 64 entries per node), and
    one global heap collection for variable-length attribute data.  ``save`` streams the file
    (object headers, then every chunk compressed one at a time).

        w = H5Writer()
        g = w.group(w.root, "posterior")
        d = w.dataset(g, "tau1", array, fill=np.nan)
        w.attr(d, "units", "yr")
        w.save(path)

    Attribute values: str (fixed-length string; nul=True adds the terminating NUL to the
    size, as the dimension-scale API writes CLASS / NAME), numbers / numpy arrays (their
    dtype), ("objref_vlen", [[handle, ...], ...]) (one variable-length sequence of object
    references per element: DIMENSION_LIST) and ("reflist", [(handle, index), ...])
    (compound {dataset: object reference, dimension: int32}: REFERENCE_LIST)."""

    def __init__(self, compress=True, level=4):
        self.objs = {}
        self.order = []
        self.compress, self.level = compress, level
        self.root = self._new("group")

    def _new(self, kind, **kw):
        h = len(self.order)
        self.objs[h] = dict(kind=kind, links=[], attrs=[], **kw)
        self.order.append(h)
        return h

    def group(self, parent, name):
        h = self._new("group")
        self.objs[parent]["links"].append((name, h))
        return h

    def dataset(self, parent, name, arr, fill=None):
        arr = np.ascontiguousarray(arr)
        if arr.dtype.kind not in "iuf" or arr.ndim == 0:
            raise ValueError("numeric arrays of rank >= 1 only")
        arr = arr.astype(arr.dtype.newbyteorder("<"))
        h = self._new("dataset", arr=arr, fill=fill)
        self.objs[parent]["links"].append((name, h))
        return h

    def attr(self, h, name, value, nul=False):
        self.objs[h]["attrs"].append((name, value, nul))

    # -------------------------------------------------------------- encoding
    def _attr_msg(self, name, value, nul, ctx):
        nb = name.encode() + b"\0"
        if isinstance(value, tuple) and value[0] == "objref_vlen":
            rows = value[1]
            dt = _dtype_msg("vlen", base=_dtype_msg("objref"))
            ds = _dataspace_msg((len(rows),))
            data = b""
            for refs in rows:
                ctx["gheap"].append(b"".join(struct.pack("<Q", ctx["addr"](r)) for r in refs))
                data += struct.pack("<IQI", len(refs), ctx["gh_addr"], len(ctx["gheap"]))
        elif isinstance(value, tuple) and value[0] == "reflist":
            rows = value[1]
            mt = [("dataset", 0, _dtype_msg("objref")), ("dimension", 8, _dtype_msg("int", 4))]
            dt = _dtype_msg("compound", size=12, members=mt)
            ds = _dataspace_msg((len(rows),))
            data = b"".join(struct.pack("<Qi", ctx["addr"](r), d) for r, d in rows)
        elif isinstance(value, str):
            s = value.encode() + (b"\0" if nul else b"")
            if not s:
                s = b"\0"
            dt = _dtype_msg("string", size=len(s))
            ds = _dataspace_msg(None)
            data = s
        else:
            a = np.asarray(value)
            if a.dtype.kind == "f":
                a = a.astype("<f%d" % a.dtype.itemsize)
                dt = _dtype_msg("float", size=a.dtype.itemsize)
            elif a.dtype.kind in "iu":
                a = a.astype(a.dtype.newbyteorder("<"))
                dt = _dtype_msg("int", size=a.dtype.itemsize, signed=a.dtype.kind == "i")
            else:
                raise ValueError("attribute %r: unsupported value %r" % (name, value))
            ds = _dataspace_msg(None if a.ndim == 0 else a.shape)
            data = a.tobytes()
        return struct.pack("<BBHHHB", 3, 0, len(nb), len(dt), len(ds), 0) + nb + dt + ds + data

    @staticmethod
    def _ohdr(msgs):
        """Version-2 object header: 4-byte chunk size, no times, no creation order."""
        body = b"".join(struct.pack("<BHB", t, len(d), 0) + d for t, d in msgs)
        blob = b"OHDR" + struct.pack("<BBI", 2, 0x02, len(body)) + body
        return blob + struct.pack("<I", lookup3(blob))

    @staticmethod
    def _link_msg(name, addr):
        nb = name.encode()
        if len(nb) > 255:
            raise ValueError("link name too long")
        return struct.pack("<BBB", 1, 0x00, len(nb)) + nb + struct.pack("<Q", addr)

    def _chunk_list(self, h):
        """Offsets (row-major order) of the dataset's chunks; none for a zero-size array."""
        arr = self.objs[h]["arr"]
        if arr.size == 0:
            return []
        cd = chunk_dims(arr.shape, arr.dtype.itemsize)
        grid = [range(0, int(d), c) for d, c in zip(arr.shape, cd)]
        return [tuple(o) for o in np.array(np.meshgrid(*grid, indexing="ij")).reshape(len(cd), -1).T]

    def _chunk_payload(self, h, off):
        """One chunk's stored bytes: the full chunk extent (edge chunks padded with the fill
        value, as the library stores them), shuffled and deflated."""
        o = self.objs[h]
        arr = o["arr"]
        cd = chunk_dims(arr.shape, arr.dtype.itemsize)
        sl = tuple(slice(a, min(a + c, d)) for a, c, d in zip(off, cd, arr.shape))
        blk = arr[sl]
        if blk.shape != cd:
            full = np.full(cd, o["fill"] if o["fill"] is not None else 0, dtype=arr.dtype)
            full[tuple(slice(0, n) for n in blk.shape)] = blk
            blk = full
        es = arr.dtype.itemsize
        sh = np.frombuffer(np.ascontiguousarray(blk).tobytes(), np.uint8).reshape(-1, es).T.tobytes()   # shuffle
        return zlib.compress(sh, self.level)

    def _payloads(self, work):
        """(h, off, payload) for the (dataset, chunk offset) pairs of ``work``, in order, deflated
        on a few threads (zlib releases the GIL: the compression is ~60 % of a trace write) with
        at most ``2 * threads`` payloads held at a time.  Same bytes as one by one."""
        import concurrent.futures as cf
        try:
            nt = len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            nt = os.cpu_count() or 1
        nt = max(1, min(8, nt, len(work)))
        if nt == 1:
            for h, off in work:
                yield h, off, self._chunk_payload(h, off)
            return
        with cf.ThreadPoolExecutor(max_workers=nt) as ex:
            pending = []
            it = iter(work)
            for h, off in it:
                pending.append((h, off, ex.submit(self._chunk_payload, h, off)))
                if len(pending) >= 2 * nt:
                    break
            for h, off in it:
                hh, oo, fu = pending.pop(0)
                yield hh, oo, fu.result()
                pending.append((h, off, ex.submit(self._chunk_payload, h, off)))
            for hh, oo, fu in pending:
                yield hh, oo, fu.result()

    def _messages(self, h, ctx):
        o = self.objs[h]
        msgs = []
        if o["kind"] == "group":
            msgs.append((0x02, struct.pack("<BB", 0, 0) + struct.pack("<QQ", UNDEF, UNDEF)))   # link info: compact
            msgs.append((0x0A, struct.pack("<BB", 0, 0)))                                      # group info
            for name, c in o["links"]:
                msgs.append((0x06, self._link_msg(name, ctx["addr"](c))))
        else:
            arr = o["arr"]
            kind = "float" if arr.dtype.kind == "f" else "int"
            msgs.append((0x01, _dataspace_msg(arr.shape, maxdims=True)))
            msgs.append((0x03, _dtype_msg(kind, size=arr.dtype.itemsize, signed=arr.dtype.kind == "i")))
            alloc = 3 if self.compress else 1                 # incremental (chunked) / early
            if o["fill"] is None:
                msgs.append((0x05, struct.pack("<BB", 3, alloc | (2 << 2))))
            else:
                fv = np.asarray(o["fill"], dtype=arr.dtype).tobytes()
                msgs.append((0x05, struct.pack("<BBI", 3, alloc | (2 << 2) | 0x20, len(fv)) + fv))
            da = ctx["data"].get(h, UNDEF)
            if self.compress:
                es = arr.dtype.itemsize
                msgs.append((0x0B, struct.pack("<BB", 2, 2) + struct.pack("<HHHI", 2, 1, 1, es)
                             + struct.pack("<HHHI", 1, 1, 1, self.level)))
                dims = b"".join(struct.pack("<I", int(x)) for x in chunk_dims(arr.shape, es)) + struct.pack("<I", es)
                msgs.append((0x08, struct.pack("<BBB", 3, 2, arr.ndim + 1) + struct.pack("<Q", ctx["btree"].get(h, UNDEF))
                             + dims))
            else:
                msgs.append((0x08, struct.pack("<BB", 3, 1) + struct.pack("<QQ", da, arr.nbytes)))
        for name, v, nul in o["attrs"]:
            msgs.append((0x0C, self._attr_msg(name, v, nul, ctx)))
        return msgs

    def _key(self, h, off, size):
        """A chunk B-tree key: stored size, filter mask 0, the chunk's offsets and 0 for the
        element dimension."""
        return struct.pack("<II", size, 0) + b"".join(struct.pack("<Q", int(x)) for x in off) + struct.pack("<Q", 0)

    def _end_key(self, h, off):
        """The key after chunk ``off`` (the node's right key): its offsets plus the chunk
        dimensions, element dimension included (the library's scaled offsets + 1, times the
        chunk dims; for a one-chunk dataset: its shape and the element size)."""
        arr = self.objs[h]["arr"]
        cd = chunk_dims(arr.shape, arr.dtype.itemsize) + (arr.dtype.itemsize,)
        return struct.pack("<II", 0, 0) + b"".join(struct.pack("<Q", int(o) + int(c)) for o, c in zip(tuple(off) + (0,), cd))

    def _node_size(self, h):
        """A v1 B-tree node at full capacity (2K children, 2K + 1 keys), as the library reads it."""
        ksz = 8 + 8 * (self.objs[h]["arr"].ndim + 1)
        return 24 + 2 * _CHUNK_K * 8 + (2 * _CHUNK_K + 1) * ksz

    @staticmethod
    def _tree_shape(n):
        """Node counts per level, leaves first, for n chunks (2K children per node)."""
        levels = []
        while True:
            n = max(1, -(-n // (2 * _CHUNK_K)))
            levels.append(n)
            if n == 1:
                return levels

    def _btree_nodes(self, h, node_addr, chunks):
        """The chunk index of a dataset: [(address, node bytes)].  chunks: [(offsets, address,
        stored size)] in row-major order; node_addr: the addresses of its nodes, leaves first
        (level by level, as _tree_shape counts them), the root last."""
        full = self._node_size(h)
        out = []
        # level 0: chunk entries; entries of a level above: (first key, right key, address).
        # A node's right key (the bound after its last child) is its right sibling's first key,
        # as the library's node splits share that key; the last node of a level ends with the
        # end key of the dataset's last chunk.
        ents = [(self._key(h, o, sz), self._end_key(h, o), a) for o, a, sz in chunks]
        k = 0
        for level, n in enumerate(self._tree_shape(len(chunks))):
            groups = [ents[i * 2 * _CHUNK_K:(i + 1) * 2 * _CHUNK_K] for i in range(n)]
            addrs = node_addr[k:k + n]
            k += n
            nxt = []
            for i, g in enumerate(groups):
                left = addrs[i - 1] if i > 0 else UNDEF
                right = addrs[i + 1] if i + 1 < n else UNDEF
                rkey = groups[i + 1][0][0] if i + 1 < n else g[-1][1]
                node = b"TREE" + struct.pack("<BBH", 1, level, len(g)) + struct.pack("<QQ", left, right)
                for key, _, a in g:
                    node += key + struct.pack("<Q", a)
                node += rkey
                out.append((addrs[i], node + b"\0" * (full - len(node))))
                nxt.append((g[0][0], rkey, addrs[i]))
            ents = nxt
        return out

    def _layout(self):
        """Pass 1: the sizes of every object header and of the global heap; returns their
        address plan (datasets' storage is placed by ``save`` as it streams it)."""
        O = 8
        sb_size = 8 + 4 + 4 * O + 4
        ctx = {"addr": lambda x: 0, "gh_addr": 0, "gheap": [], "data": {}, "btree": {}}
        sizes = {h: len(self._ohdr(self._messages(h, ctx))) for h in self.order}
        gh_blobs = [len(x) for x in ctx["gheap"]]
        addr, p = {}, sb_size
        for h in self.order:
            addr[h] = p
            p += sizes[h]
        gh_addr = p
        gh_used = 16 + sum(16 + n + (-n % 8) for n in gh_blobs)
        gh_size = max(4096, gh_used + 16) if gh_blobs else 0
        return {"sb_size": sb_size, "sizes": sizes, "addr": addr, "gh_addr": gh_addr, "gh_size": gh_size,
                "end": p + gh_size}

    def save(self, path_or_file):
        """Write the file (a path or a seekable binary file object).  Datasets are streamed
        after the metadata: a contiguous one as its bytes, a chunked one as its B-tree nodes
        (their count follows from the chunk count) then each chunk, compressed on a few
        threads ahead of the writes (a bounded window of payloads held, _payloads) and written
        in order; the superblock and object headers,
        whose sizes pass 1 fixed, are written last, when every address is known."""
        import io
        lay = self._layout()
        f = open(path_or_file, "wb") if isinstance(path_or_file, str) else path_or_file
        try:
            O = 8
            addr = lay["addr"]
            base = f.tell() if not isinstance(path_or_file, str) else 0
            if base:
                raise H5Error("H5Writer.save: the file object must be positioned at 0")

            def put(a, blob):
                f.seek(a)
                f.write(blob)
            p = lay["end"]
            data, btree = {}, {}
            # every chunk of every compressed dataset, in the order they are written below
            stream = self._payloads([(h, off) for h in self.order
                                     if self.compress and self.objs[h]["kind"] == "dataset" for off in self._chunk_list(h)])
            for h in self.order:
                if self.objs[h]["kind"] != "dataset":
                    continue
                arr = self.objs[h]["arr"]
                if not self.compress:
                    p = (p + 7) // 8 * 8
                    data[h] = p
                    put(p, np.ascontiguousarray(arr).tobytes())
                    p += arr.nbytes
                    continue
                offs = self._chunk_list(h)
                if not offs:              # nothing stored: the B-tree address stays undefined
                    continue
                nodes = []
                for _ in range(sum(self._tree_shape(len(offs)))):
                    nodes.append(p)
                    p += self._node_size(h)
                ch = []
                for off in offs:
                    hh, oo, pl = next(stream)
                    assert hh == h and oo == off
                    p = (p + 7) // 8 * 8
                    put(p, pl)
                    ch.append((off, p, len(pl)))
                    p += len(pl)
                for na, node in self._btree_nodes(h, nodes, ch):
                    put(na, node)
                btree[h] = nodes[-1]      # the root
            eof = p
            ctx = {"addr": lambda x: addr[x], "gh_addr": lay["gh_addr"], "gheap": [], "data": data, "btree": btree}
            sb = _SIG + struct.pack("<BBBB", 2, O, O, 0) + struct.pack("<QQQQ", 0, UNDEF, eof, addr[self.root])
            put(0, sb + struct.pack("<I", lookup3(sb)))
            for h in self.order:
                blob = self._ohdr(self._messages(h, ctx))
                if len(blob) != lay["sizes"][h]:
                    raise H5Error("object header size changed between passes")
                put(addr[h], blob)
            gh_size = lay["gh_size"]
            if gh_size:
                body = b"".join(struct.pack("<HHIQ", i + 1, 1, 0, len(x)) + x + b"\0" * (-len(x) % 8)
                                for i, x in enumerate(ctx["gheap"]))
                col = b"GCOL" + struct.pack("<B3xQ", 1, gh_size) + body
                free = gh_size - len(col)
                if free >= 16:
                    col += struct.pack("<HHIQ", 0, 0, 0, free)          # the free-space object
                put(lay["gh_addr"], col + b"\0" * (gh_size - len(col)))
            f.seek(0, io.SEEK_END)
            if f.tell() < eof:            # (the end of file the superblock records)
                f.seek(eof - 1)
                f.write(b"\0")
        finally:
            if isinstance(path_or_file, str):
                f.close()
        return path_or_file

    def tobytes(self):
        import io
        b = io.BytesIO()
        self.save(b)
        return b.getvalue()


# ------------------------------------------------------------------ netCDF-4 on top
# netCDF's default fill values of the signed integer types (netcdf.h NC_FILL_BYTE / INT / INT64),
# which netCDF records in the HDF5 fill-value message of integer variables
_NC_FILL = {1: np.int8(-127), 4: np.int32(-2147483647), 8: np.int64(-9223372036854775806)}


def write_netcdf4(path, groups, root_attrs=None, compress=True):
    """A netCDF-4 file of ``groups``: {group: {"attrs": {...}, "dims": {name: coord array},
    "vars": {name: (dims tuple, array, attrs dict)}}} -- the layout az.to_netcdf writes
    (ArviZ 0.11.4 through netCDF 4.8.1): every dimension is a coordinate variable and an
    HDF5 dimension scale (CLASS, NAME, REFERENCE_LIST), every variable carries its
    DIMENSION_LIST, and netCDF's _Netcdf4Dimid / _Netcdf4Coordinates (dimension ids are
    numbered across the file in group order)."""
    w = H5Writer(compress=compress)
    w.attr(w.root, "_NCProperties", (root_attrs or {}).get("_NCProperties", "version=2,ngrtd_h5lite=1"))
    dimid = 0
    for gname, g in groups.items():
        gh = w.group(w.root, gname)
        for k, v in g.get("attrs", {}).items():
            w.attr(gh, k, v)
        ids, dh = {}, {}
        for dname, coord in g["dims"].items():
            ids[dname] = dimid
            dimid += 1
            coord = np.asarray(coord)
            dh[dname] = w.dataset(gh, dname, coord, fill=_NC_FILL.get(coord.dtype.itemsize)
                                  if coord.dtype.kind == "i" else None)
        vh, refs = {}, {d: [] for d in g["dims"]}
        for vname, (dims, arr, attrs) in g["vars"].items():
            arr = np.asarray(arr)
            if tuple(arr.shape) != tuple(len(g["dims"][d]) for d in dims):
                raise ValueError("%s/%s: shape %s does not match dims %s" % (gname, vname, arr.shape, dims))
            fill = np.nan if arr.dtype.kind == "f" else _NC_FILL.get(arr.dtype.itemsize)
            h = w.dataset(gh, vname, arr, fill=fill)
            vh[vname] = h
            w.attr(h, "_Netcdf4Coordinates", np.array([ids[d] for d in dims], dtype=np.int32))
            if arr.dtype.kind == "f":
                w.attr(h, "_FillValue", np.array([np.nan]))
            for k, v in (attrs or {}).items():
                w.attr(h, k, v)
            w.attr(h, "DIMENSION_LIST", ("objref_vlen", [[dh[d]] for d in dims]))
            if len(dims) > 1:        # as netCDF 4.8.1 writes them (the shipped traces)
                w.attr(h, "_Netcdf4Dimid", np.int32(ids[dims[0]]))
            for i, d in enumerate(dims):
                refs[d].append((h, i))
        for dname, h in dh.items():
            w.attr(h, "_Netcdf4Coordinates", np.array([ids[dname]], dtype=np.int32))
            w.attr(h, "CLASS", "DIMENSION_SCALE", nul=True)
            w.attr(h, "NAME", dname, nul=True)
            w.attr(h, "_Netcdf4Dimid", np.int32(ids[dname]))
            if refs[dname]:
                w.attr(h, "REFERENCE_LIST", ("reflist", refs[dname]))
    return w.save(path)


def read_netcdf4(path):
    """{group: {"attrs", "dims": {name: coord}, "vars": {name: (dims, array, attrs)}}} of a
    netCDF-4 file (dimension names resolved through each variable's DIMENSION_LIST)."""
    r = H5Reader(path)
    out = {"attrs": r.attrs(r.root)}
    for gname, ga in r.links(r.root).items():
        if r.is_dataset(ga):
            continue
        links = r.links(ga)
        by_addr = {}
        g = {"attrs": r.attrs(ga), "dims": {}, "vars": {}}
        for name, a in links.items():
            at = r.attrs(a)
            if at.get("CLASS") == "DIMENSION_SCALE":
                g["dims"][name] = r.read(a)
                by_addr[a] = name
        for name, a in links.items():
            if a in by_addr:
                continue
            at = r.attrs(a)
            dl = at.pop("DIMENSION_LIST", None)
            dims = tuple(by_addr[int(x[0])] for x in dl) if dl is not None else ()
            for k in ("_Netcdf4Coordinates", "_Netcdf4Dimid"):
                at.pop(k, None)
            g["vars"][name] = (dims, r.read(a), at)
        out[gname] = g
    return out


def structure(path):
    """The comparable structure of a netCDF-4 file: {group: {"attrs": {name: type},
    "vars": {name: {"dtype", "dims", "attrs": {name: type}, "filters"}}}} (+ "/" for the
    root attributes) -- names, types, dimension names and storage filters, not values."""
    r = H5Reader(path)
    out = {"/": {k: v[0].describe() for k, v in r.attrs(r.root, raw=True).items()}}
    for gname, ga in r.links(r.root).items():
        if r.is_dataset(ga):
            continue
        links = r.links(ga)
        names = {a: n for n, a in links.items()}
        g = {"attrs": {k: v[0].describe() for k, v in r.attrs(ga, raw=True).items()}, "vars": {}}
        for name, a in links.items():
            at = r.attrs(a, raw=True)
            dt, dims, _, filters = r.dataset_info(a)
            dl = at.get("DIMENSION_LIST")
            dnames = [names.get(int(x[0]), "?") for x in dl[2]] if dl is not None else [name]
            g["vars"][name] = {"dtype": dt.describe(), "dims": dnames, "filters": [f[0] for f in filters],
                               "attrs": {k: v[0].describe() for k, v in at.items()}}
        out[gname] = g
    return out
