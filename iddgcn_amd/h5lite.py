"""Minimal HDF5 reader and writer for Keras weight files, without h5py.

The reference saves and loads its weights as Keras-h5 files (IDDGCN.py:181-199 SaveWeightsCallback,
IDDGCN_eval.py:46-47 load_weights).  h5py is not importable on this image's main Python, so this
module implements the part of the HDF5 file format (spec version 2/3, "earliest" layout as written by
h5py for Keras) those files use:

  superblock v0/v1, object headers v1 (+ continuation blocks), old-style groups (symbol-table message,
  v1 B-tree of group nodes, local heap, SNOD symbol-table nodes), datasets with a v1/v2 dataspace,
  fixed-point / IEEE-float / fixed-length-string datatypes and a v3 compact or contiguous layout,
  and v1/v2/v3 attribute messages.

Anything else (chunked or filtered datasets, v2 object headers, new-style link groups, variable-length
strings) raises H5Error naming the unsupported feature.  Reading is pure parsing: nothing in the file
is executed or unpickled.

The writer produces the same subset (what h5py writes with libver="earliest"): a file Keras / h5py
read back (checked in tests/test_h5lite.py when the image's h5py interpreter is present).
"""
import struct

import numpy as np


class H5Error(ValueError):
    pass


_SIG = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF


# =============================================================================================
# reader
# =============================================================================================
class _Reader:
    def __init__(self, data):
        self.d = data
        if data[:8] != _SIG:
            raise H5Error("not an HDF5 file (bad signature)")
        ver = data[8]
        if ver not in (0, 1):
            raise H5Error(f"superblock version {ver} unsupported (only 0/1, h5py libver='earliest')")
        self.so, self.sl = data[13], data[14]
        if self.so != 8 or self.sl != 8:
            raise H5Error("only 8-byte offsets/lengths are supported")
        p = 24 if ver == 0 else 28
        p += 8 * 4                                        # base, free-space, EOF, driver addresses
        self.root = self._symbol_entry(p)[1]

    # -- primitives --
    def u(self, off, n):
        return int.from_bytes(self.d[off:off + n], "little")

    def _symbol_entry(self, p):
        name_off, hdr = self.u(p, 8), self.u(p + 8, 8)
        return name_off, hdr

    def _cstr(self, off):
        end = self.d.index(b"\x00", off)
        return self.d[off:end].decode("utf-8")

    # -- object headers --
    def messages(self, addr):
        d = self.d
        if d[addr:addr + 4] == b"OHDR":
            raise H5Error("version-2 object headers unsupported")
        if d[addr] != 1:
            raise H5Error(f"object header version {d[addr]} unsupported")
        nmsg, size = self.u(addr + 2, 2), self.u(addr + 8, 4)
        blocks = [(addr + 16, size)]
        out = []
        while blocks:
            start, length = blocks.pop(0)
            p = start
            while p + 8 <= start + length and len(out) < nmsg:
                mtype, msize, flags = self.u(p, 2), self.u(p + 2, 2), d[p + 4]
                body = p + 8
                if flags & 0x02:
                    raise H5Error("shared header messages unsupported")
                if mtype == 0x10:                          # continuation
                    blocks.append((self.u(body, 8), self.u(body + 8, 8)))
                out.append((mtype, body, msize))
                p = body + msize
        return out

    def attrs(self, addr):
        res = {}
        for mtype, body, _ in self.messages(addr):
            if mtype == 0x0C:
                name, value = self._attribute(body)
                res[name] = value
        return res

    def _attribute(self, p):
        ver = self.d[p]
        nsz, tsz, ssz = self.u(p + 2, 2), self.u(p + 4, 2), self.u(p + 6, 2)
        q = p + 8 + (1 if ver == 3 else 0)
        pad = (lambda n: (n + 7) & ~7) if ver == 1 else (lambda n: n)
        name = self.d[q:q + nsz].split(b"\x00")[0].decode("utf-8")
        q += pad(nsz)
        dt = self._datatype(q)
        q += pad(tsz)
        shape = self._dataspace(q)
        q += pad(ssz)
        return name, self._decode(q, dt, shape)

    def _datatype(self, p):
        cls, ver = self.d[p] & 0x0F, self.d[p] >> 4
        bits = self.d[p + 1:p + 4]
        size = self.u(p + 4, 4)
        if cls == 0:                                       # fixed-point
            if bits[0] & 1:
                raise H5Error("big-endian integers unsupported")
            return np.dtype(f"<{'i' if bits[0] & 0x08 else 'u'}{size}")
        if cls == 1:                                       # IEEE float
            if bits[0] & 1:
                raise H5Error("big-endian floats unsupported")
            return np.dtype(f"<f{size}")
        if cls == 3:                                       # fixed-length string
            return np.dtype(f"S{size}")
        if cls == 9 and (bits[0] & 0x0F) == 1:             # variable-length string (global heap)
            return "vlen-str"
        raise H5Error(f"datatype class {cls} (v{ver}) unsupported")

    def _dataspace(self, p):
        ver, ndim, flags = self.d[p], self.d[p + 1], self.d[p + 2]
        if ver == 1:
            q = p + 8
        elif ver == 2:
            if self.d[p + 3] == 2:                         # null dataspace
                return None
            q = p + 4
        else:
            raise H5Error(f"dataspace version {ver} unsupported")
        return tuple(self.u(q + 8 * i, 8) for i in range(ndim))

    def _decode(self, p, dt, shape):
        if shape is None:
            return None
        n = int(np.prod(shape)) if shape else 1
        if isinstance(dt, str):                            # vlen strings: (len, collection, index)
            vals = []
            for k in range(n):
                q = p + 16 * k
                vals.append(self._global_heap_object(self.u(q + 4, 8), self.u(q + 12, 4)).decode("utf-8"))
            a = np.array(vals, dtype=object)
        else:
            a = np.frombuffer(self.d, dtype=dt, count=n, offset=p).copy()
        return a.reshape(shape) if shape else a[0]

    def _global_heap_object(self, coll, index):
        d = self.d
        if d[coll:coll + 4] != b"GCOL":
            raise H5Error("bad global heap collection")
        end = coll + self.u(coll + 8, 8)
        p = coll + 16
        while p + 16 <= end:
            idx, size = self.u(p, 2), self.u(p + 8, 8)
            if idx == 0:
                break
            if idx == index:
                return bytes(d[p + 16:p + 16 + size])
            p += 16 + ((size + 7) & ~7)
        raise H5Error(f"global heap object {index} not found")

    # -- groups --
    def children(self, addr):
        for mtype, body, _ in self.messages(addr):
            if mtype == 0x11:                              # symbol table message
                btree, heap = self.u(body, 8), self.u(body + 8, 8)
                return self._group_entries(btree, heap)
            if mtype in (0x02, 0x06, 0x0A):
                raise H5Error("new-style (link message) groups unsupported")
        return None                                        # not a group

    def _group_entries(self, btree, heap):
        d = self.d
        if d[heap:heap + 4] != b"HEAP":
            raise H5Error("bad local heap")
        data_seg = self.u(heap + 24, 8)
        out = {}

        def node(addr):
            if d[addr:addr + 4] != b"TREE":
                raise H5Error("bad B-tree node")
            ntype, level, used = d[addr + 4], d[addr + 5], self.u(addr + 6, 2)
            if ntype != 0:
                raise H5Error("not a group B-tree")
            p = addr + 24
            for _ in range(used):
                child = self.u(p + 8, 8)                    # key (8) then child address (8)
                p += 16
                if level > 0:
                    node(child)
                else:
                    snod(child)

        def snod(addr):
            if d[addr:addr + 4] != b"SNOD":
                raise H5Error("bad symbol table node")
            n = self.u(addr + 6, 2)
            p = addr + 8
            for _ in range(n):
                name_off, hdr = self._symbol_entry(p)
                out[self._cstr(data_seg + name_off)] = hdr
                p += 40

        node(btree)
        return out

    # -- datasets --
    def dataset(self, addr):
        dt = shape = None
        layout = None
        for mtype, body, _ in self.messages(addr):
            if mtype == 0x01:
                shape = self._dataspace(body)
            elif mtype == 0x03:
                dt = self._datatype(body)
            elif mtype == 0x08:
                layout = body
            elif mtype == 0x0B:
                raise H5Error("filtered (compressed) datasets unsupported")
        if dt is None or layout is None:
            raise H5Error("object is not a dataset")
        ver, cls = self.d[layout], self.d[layout + 1]
        if ver != 3:
            raise H5Error(f"data layout message version {ver} unsupported")
        if cls == 0:                                       # compact
            return self._decode(layout + 4, dt, shape)
        if cls == 1:                                       # contiguous
            addr = self.u(layout + 2, 8)
            if addr == UNDEF:
                return np.zeros(shape, dt)
            return self._decode(addr, dt, shape)
        raise H5Error("chunked datasets unsupported")


class Node:
    """A group or dataset of an H5File (h5py-like: node[path], node.attrs, np.asarray(dataset))."""

    def __init__(self, reader, addr, name):
        self._r, self._addr, self.name = reader, addr, name
        self._kids = reader.children(addr)

    @property
    def attrs(self):
        return self._r.attrs(self._addr)

    def is_group(self):
        return self._kids is not None

    def keys(self):
        return list(self._kids or {})

    def __getitem__(self, path):
        node = self
        for part in [p for p in path.split("/") if p]:
            if not node.is_group() or part not in node._kids:
                raise KeyError(f"{path!r} not found under {self.name!r}")
            node = Node(self._r, node._kids[part], f"{node.name.rstrip('/')}/{part}")
        return node

    def __array__(self, dtype=None, copy=None):
        a = self._r.dataset(self._addr)
        return a if dtype is None else a.astype(dtype)

    def read(self):
        return self._r.dataset(self._addr)


def open_file(path):
    """Parse an HDF5 file (the subset above) into a root Node."""
    with open(path, "rb") as f:
        data = f.read()
    r = _Reader(data)
    return Node(r, r.root, "/")


# =============================================================================================
# writer (superblock v0, v1 object headers, symbol-table groups, contiguous datasets)
# =============================================================================================
def _pad8(b):
    return b + b"\x00" * ((-len(b)) % 8)


class _Writer:
    K_LEAF = 4          # group leaf node K: a SNOD holds up to 2K entries
    K_INT = 16

    def __init__(self):
        self.buf = bytearray(b"\x00" * 96)            # superblock + root symbol entry, patched later
        self.fix = []

    def alloc(self, b):
        off = len(self.buf)
        self.buf += _pad8(bytes(b))
        return off

    @staticmethod
    def msg(mtype, body, flags=0):
        body = _pad8(body)
        return struct.pack("<HHB3x", mtype, len(body), flags) + body

    @staticmethod
    def dtype_msg(dt):
        dt = np.dtype(dt)
        if dt.kind == "f":
            if dt.itemsize == 4:
                props = struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
            else:
                props = struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
            # class 1 v1; bits: byte order LE, pad 0, mantissa normalization "implied" (2 << 4),
            # sign bit position 31 / 63
            bits = bytes([0x20, dt.itemsize * 8 - 1, 0])
            return bytes([0x11]) + bits + struct.pack("<I", dt.itemsize) + props
        if dt.kind in "iu":
            bits = bytes([0x08 if dt.kind == "i" else 0x00, 0, 0])
            return bytes([0x10]) + bits + struct.pack("<I", dt.itemsize) + struct.pack("<HH", 0, dt.itemsize * 8)
        if dt.kind == "S":
            return bytes([0x13, 0x00, 0, 0]) + struct.pack("<I", dt.itemsize)   # null-terminated, ASCII
        raise H5Error(f"cannot write dtype {dt}")

    @staticmethod
    def space_msg(shape):
        if shape == ():
            return struct.pack("<BBBx4x", 1, 0, 0)
        return struct.pack("<BBBx4x", 1, len(shape), 0) + b"".join(struct.pack("<Q", n) for n in shape)

    def attr_msg(self, name, value):
        a = np.asarray(value)
        if a.dtype.kind == "U":
            a = np.char.encode(a, "utf-8")
        if a.dtype.kind == "S" and a.dtype.itemsize == 0:
            a = a.astype("S1")
        nm = name.encode() + b"\x00"
        dt, sp = self.dtype_msg(a.dtype), self.space_msg(a.shape)
        body = struct.pack("<BxHHH", 1, len(nm), len(dt), len(sp)) + _pad8(nm) + _pad8(dt) + _pad8(sp)
        return self.msg(0x0C, body + np.ascontiguousarray(a).tobytes())

    def object_header(self, msgs):
        blob = b"".join(msgs)
        hdr = struct.pack("<BxHII", 1, len(msgs), 1, len(blob)) + b"\x00" * 4
        return self.alloc(hdr + blob)

    def dataset(self, arr, attrs=None):
        a = np.ascontiguousarray(arr)
        data_addr = self.alloc(a.tobytes())
        layout = struct.pack("<BBQQ", 3, 1, data_addr, a.nbytes)
        fill = struct.pack("<BBBB", 2, 2, 2, 0)       # fill value message v2: alloc late, write never, undefined
        msgs = [self.msg(0x01, self.space_msg(a.shape)), self.msg(0x03, self.dtype_msg(a.dtype), flags=1),
                self.msg(0x05, fill, flags=1), self.msg(0x08, layout)]
        msgs += [self.attr_msg(k, v) for k, v in (attrs or {}).items()]
        return self.object_header(msgs)

    def group(self, children, attrs=None):
        """children: list of (name, object header address), any order (stored sorted by name)."""
        children = sorted(children, key=lambda c: c[0].encode())
        # local heap: offset 0 is the empty string
        heap_data = bytearray(b"\x00" * 8)
        offs = []
        for name, _ in children:
            offs.append(len(heap_data))
            heap_data += _pad8(name.encode() + b"\x00")
        heap_data += b"\x00" * 16                      # a free block for h5py-friendliness
        free_off = len(heap_data) - 16
        heap_data[free_off:free_off + 16] = struct.pack("<QQ", 1, 16)
        data_addr = self.alloc(heap_data)
        heap = b"HEAP" + struct.pack("<B3xQQQ", 0, len(heap_data), free_off, data_addr)
        heap_addr = self.alloc(heap)
        # symbol table nodes, 2K entries each, and one level-0 B-tree over them
        cap = 2 * self.K_LEAF
        snods = []
        for s in range(0, max(len(children), 1), cap):
            chunk = list(zip(offs, children))[s:s + cap]
            ents = b"".join(struct.pack("<QQI4x16x", o, a, 0) for o, (_, a) in chunk)
            ents += b"\x00" * (40 * (cap - len(chunk)))
            snods.append((self.alloc(b"SNOD" + struct.pack("<BxH", 1, len(chunk)) + ents),
                          chunk[-1][0] if chunk else 0))
        if len(snods) > 2 * self.K_INT:
            raise H5Error("group too large for a single B-tree node")
        keys = b"".join(struct.pack("<QQ", 0 if i == 0 else snods[i - 1][1], addr)
                        for i, (addr, _) in enumerate(snods))
        keys += struct.pack("<Q", snods[-1][1])
        keys += b"\x00" * (16 * (2 * self.K_INT - len(snods)))
        btree = b"TREE" + struct.pack("<BBHQQ", 0, 0, len(snods), UNDEF, UNDEF) + keys
        btree_addr = self.alloc(btree)
        msgs = [self.msg(0x11, struct.pack("<QQ", btree_addr, heap_addr))]
        msgs += [self.attr_msg(k, v) for k, v in (attrs or {}).items()]
        return self.object_header(msgs), btree_addr, heap_addr

    def finish(self, root):
        hdr_addr, btree, heap = root
        sb = _SIG + struct.pack("<BBBBBBBB", 0, 0, 0, 0, 0, 8, 8, 0)
        sb += struct.pack("<HHI", self.K_LEAF, self.K_INT, 0)
        sb += struct.pack("<QQQQ", 0, UNDEF, len(self.buf), UNDEF)
        sb += struct.pack("<QQI4xQQ", 0, hdr_addr, 1, btree, heap)
        self.buf[:len(sb)] = sb
        return bytes(self.buf)


def write_file(path, tree, attrs=None):
    """Write a nested dict {name: ndarray | (dict, attrs) | dict} as an HDF5 file; `attrs` are the
    root attributes.  A group value may be a dict or a (dict, attrs) pair."""
    w = _Writer()

    def build(node, node_attrs):
        kids = []
        for name, v in node.items():
            if isinstance(v, tuple):
                sub, sub_attrs = v
                kids.append((name, build(sub, sub_attrs)[0]))
            elif isinstance(v, dict):
                kids.append((name, build(v, None)[0]))
            else:
                kids.append((name, w.dataset(v)))
        return w.group(kids, node_attrs)

    data = w.finish(build(tree, attrs))
    with open(path, "wb") as f:
        f.write(data)
