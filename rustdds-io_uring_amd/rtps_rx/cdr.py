"""Sample types for the batch CDR decode.

The reference decodes one sample at a time through serde:
  SimpleDataReader::deserialize_with        io_uring/dds/with_key/simpledatareader.rs:137-160
  -> CDRDeserializerAdapter::from_bytes_with dds/adapters.rs:128-139, serialization/cdr_adapters.rs:96-100
  -> deserialize_from_cdr_with_decoder_and_rep_id  cdr_adapters.rs:246-275 (cdr-encoding 0.10)
Here a `#[derive(Deserialize)]` struct becomes a `CdrType`: the flat list of
rtps_cdr_op (include/rtps_rx.h) that the GPU decodes for every DATA record of
a parsed batch, plus the numpy dtype of the fixed-layout output row.

    ShapeType = CdrType([("color", String(128)), ("x", "i32"), ("y", "i32"), ("shapesize", "i32")])

Field specs: a primitive name (PRIMS), "bool", String(cap), Seq(elem, cap),
Array(elem, n) or a nested CdrType (flattened: classic CDR aligns each
primitive to its own size from the start of the value, so nesting adds no
padding of its own).  A Seq / Array element is a primitive name (one SEQ /
ARRAY op) or any other spec -- String, Seq, Array, CdrType -- which becomes a
SEQ_BEGIN / ARRAY_BEGIN op, the element's own program and an END op (serde's
Vec<T> / [T; N] of strings, structs or sequences):

    Polygon = CdrType([("name", String(16)), ("pts", Seq(CdrType([("x", "f32"), ("y", "f32")]), 8)),
                       ("tags", Seq(String(12), 4))])
"""
import numpy as np

OP_PRIM, OP_BOOL, OP_STRING, OP_SEQ, OP_ARRAY = 1, 2, 3, 4, 5
OP_SEQ_BEGIN, OP_ARRAY_BEGIN, OP_END = 6, 7, 8
CDR_OK, CDR_NOT_DATA, CDR_BAD_ENCODING, CDR_EOF, CDR_BAD_BOOL, CDR_BAD_UTF8, CDR_TOO_LONG = range(7)
CDR_STATUS_NAMES = {0: "OK", 1: "NOT_DATA", 2: "BAD_ENCODING", 3: "EOF", 4: "BAD_BOOL", 5: "BAD_UTF8",
                    6: "TOO_LONG"}
MAX_OPS = 64
MAX_DEPTH = 4  # RTPS_CDR_MAX_DEPTH

OP_DTYPE = np.dtype([("kind", "u1"), ("size", "u1"), ("stride", "<u2"), ("count", "<u4"), ("out_off", "<u4")])
assert OP_DTYPE.itemsize == 12

# serde primitive -> numpy type.  (Rust `char` is a 4-byte code point in
# cdr-encoding and is not offered; unit enums are their u32 discriminant.)
PRIMS = {"u8": "u1", "i8": "i1", "u16": "<u2", "i16": "<i2", "u32": "<u4", "i32": "<i4",
         "f32": "<f4", "u64": "<u8", "i64": "<i8", "f64": "<f8"}


class String:
    def __init__(self, cap):
        self.cap = int(cap)


class _Composite:
    """Seq / Array: element `elem` (a primitive name or any other field spec)."""

    def __init__(self, elem, count):
        self.elem = elem
        self.prim = elem if isinstance(elem, str) and elem in PRIMS else None
        if self.prim is None:
            # a bare element spec is wrapped in a one-field struct "v" (unwrapped by to_python)
            self.wrapped = not isinstance(elem, CdrType)
            self.elem_type = CdrType([("v", elem)]) if self.wrapped else elem


class Seq(_Composite):
    def __init__(self, elem, cap):
        super().__init__(elem, cap)
        self.cap = int(cap)


class Array(_Composite):
    def __init__(self, elem, n):
        super().__init__(elem, n)
        self.n = int(n)


def _align(x, a):
    return (x + a - 1) // a * a


class CdrType:
    """Flat decode program + row layout of one sample type."""

    def __init__(self, fields):
        self.fields = list(fields)
        ops, names, formats, offsets = [], [], [], []
        self._layout = []  # (name, kind, spec) in program order, for encoders/decoders
        self.depth = 0     # SEQ_BEGIN / ARRAY_BEGIN nesting
        pos = 0

        def add(name, spec):
            nonlocal pos
            if isinstance(spec, CdrType):
                for sub_name, sub_spec in spec.fields:
                    add(f"{name}.{sub_name}", sub_spec)
                return
            # every slot is 4-aligned and a multiple of 4 bytes (include/rtps_rx.h)
            if isinstance(spec, str) and spec in PRIMS:
                dt = np.dtype(PRIMS[spec])
                kind, size, count, fmt, slot = OP_PRIM, dt.itemsize, 1, dt, _align(dt.itemsize, 4)
            elif spec == "bool":
                kind, size, count, fmt, slot = OP_BOOL, 1, 1, np.dtype("u1"), 4
            elif isinstance(spec, String):
                kind, size, count, slot = OP_STRING, 1, spec.cap, 4 + _align(spec.cap, 4)
                fmt = np.dtype([("len", "<u4")] + ([("data", f"S{_align(spec.cap, 4)}")] if spec.cap else []))
            elif isinstance(spec, (Seq, Array)) and spec.prim is None:
                et = spec.elem_type
                seq = isinstance(spec, Seq)
                count = spec.cap if seq else spec.n
                if et.row_bytes > 0xFFFF or et.depth + 1 > MAX_DEPTH:
                    raise ValueError(f"{name}: element too large or nested too deep")
                hdr = 4 if seq else 0
                fmt = np.dtype(([("n", "<u4")] if seq else []) + [("data", et.row_dtype, (count,))])
                ops.append((OP_SEQ_BEGIN if seq else OP_ARRAY_BEGIN, 0, et.row_bytes, count, pos))
                ops.extend(tuple(o) for o in et.ops.tolist())
                ops.append((OP_END, 0, 0, 0, 0))
                self.depth = max(self.depth, et.depth + 1)
                names.append(name)
                formats.append(fmt)
                offsets.append(pos)
                self._layout.append((name, OP_SEQ_BEGIN if seq else OP_ARRAY_BEGIN, spec))
                pos += hdr + count * et.row_bytes
                return
            elif isinstance(spec, Seq):
                dt = np.dtype(PRIMS[spec.prim])
                kind, size, count, slot = OP_SEQ, dt.itemsize, spec.cap, 4 + _align(dt.itemsize * spec.cap, 4)
                fmt = np.dtype([("n", "<u4")] + ([("data", dt, (spec.cap,))] if spec.cap else []))
            elif isinstance(spec, Array):
                dt = np.dtype(PRIMS[spec.prim])
                kind, size, count, slot = OP_ARRAY, dt.itemsize, spec.n, _align(dt.itemsize * spec.n, 4)
                fmt = np.dtype((dt, (spec.n,)))
            else:
                raise TypeError(f"unsupported field spec {spec!r} for {name}")
            ops.append((kind, size, 0, count, pos))
            names.append(name)
            formats.append(fmt)
            offsets.append(pos)
            self._layout.append((name, kind, spec))
            pos += slot

        for name, spec in self.fields:
            add(name, spec)
        if len(ops) > MAX_OPS:
            raise ValueError(f"{len(ops)} ops > {MAX_OPS}")
        self.row_bytes = max(pos, 4)
        self.ops = np.array(ops, dtype=OP_DTYPE)
        self.row_dtype = np.dtype({"names": names, "formats": formats, "offsets": offsets,
                                   "itemsize": self.row_bytes})

    @property
    def n_ops(self):
        return len(self.ops)

    def rows(self, raw):
        """[m, row_bytes] u8 -> structured rows."""
        return np.ascontiguousarray(raw, dtype=np.uint8).reshape(-1).view(self.row_dtype)

    def to_python(self, row):
        """One structured row -> {field: value} with str / list values."""
        out = {}
        for name, kind, spec in self._layout:
            v = row[name]
            if kind == OP_STRING:
                out[name] = v.tobytes()[4:4 + int(v["len"])].decode()
            elif kind == OP_SEQ:
                out[name] = v["data"][: int(v["n"])].tolist() if spec.cap else []
            elif kind in (OP_SEQ_BEGIN, OP_ARRAY_BEGIN):
                et = spec.elem_type
                els = v["data"][: int(v["n"])] if kind == OP_SEQ_BEGIN else v["data"]
                out[name] = [et.to_python(e)["v"] if spec.wrapped else et.to_python(e) for e in els]
            elif kind == OP_ARRAY:
                out[name] = v.tolist()
            elif kind == OP_BOOL:
                out[name] = bool(v)
            else:
                out[name] = v.item()
        return out


# The shapes-demo sample type (rtps/message_receiver.rs:1240-1248: color, x, y, size)
ShapeType = CdrType([("color", String(128)), ("x", "i32"), ("y", "i32"), ("shapesize", "i32")])

# Sample type of the C2 / T synthetic workloads' payloads (252 / 976 value bytes
# of primitives after the CDR_LE header; the trailing bytes are ignored, as
# cdr-encoding only reports bytes_consumed).
C2Sample = CdrType([("seq", "u64"), ("stamp", "f64"), ("vals", Array("f32", 58))])
TSample = CdrType([("seq", "u64"), ("stamp", "f64"), ("vals", Array("f32", 240))])
