"""f1: the heap keyed-state backend's snapshot format, read and written as data (no Java code is run, no Java object
is deserialized).  This is the host side of a checkpoint: the GPU operators' per-key-group rows (fw_snapshot_key_group
/ fw_list_snapshot_key_group) become the key-group sections a CPU HeapKeyedStateBackend restores, and a savepoint the
CPU operator wrote restores into the GPU operators.  Reference formats (paths relative to /root/reference):

  flink-streaming-java/src/test/java/org/apache/flink/streaming/util/OperatorSnapshotUtil.java:48-104
      operator snapshot file: chain index, legacy handle, raw / managed operator state, raw / managed keyed state
  flink-runtime/.../checkpoint/savepoint/SavepointV1Serializer.java:215-360
      KeyGroupsStateHandle (type 3: start key group, count, offsets) over a ByteStreamStateHandle (type 1)
  flink-runtime/.../state/KeyedBackendSerializationProxy.java:101-155
      version, key-group compression flag (v4), key serializer, the registered states' meta info
  flink-core/.../api/common/typeutils/TypeSerializerSerializationUtil.java:139-214
      serializers + config snapshots written "with resilience": offsets and a length-prefixed block, skipped here
  flink-runtime/.../state/KeyedBackendStateMetaInfoSnapshotReaderWriters.java:96-116   state type, name, serializers
  flink-runtime/.../state/heap/HeapKeyedStateBackend.java:366-383
      per key group: key group id, then per state its short id and writeMappingsInKeyGroup
  flink-runtime/.../state/heap/CopyOnWriteStateTableSnapshot.java:175-198   count, then (namespace, key, state)
  flink-streaming-java/.../api/operators/InternalTimerServiceSerializationProxy.java:91-133,
  InternalTimersSnapshotReaderWriters.java:96-160, InternalTimer.java:148-159
      raw keyed state: timer services per key group; timer = (key, namespace, timestamp)

Java-serialized serializer objects (the pre-versioned timer format writes them bare) are skipped with a structural
reader of the serialization stream grammar (class descriptors, field values, block data): it only walks the bytes.
"""
import io
import struct

from .keygroups import _i32, bit_mix

# ---------------------------------------------------------------- DataInputStream / DataOutputStream


class DataInput:
    def __init__(self, data, pos=0):
        self.b = bytes(data)
        self.pos = pos

    def take(self, n):
        if self.pos + n > len(self.b):
            raise ValueError(f"truncated stream at {self.pos} (+{n} of {len(self.b)})")
        v = self.b[self.pos:self.pos + n]
        self.pos += n
        return v

    def u8(self):
        return self.take(1)[0]

    def i8(self):
        return struct.unpack(">b", self.take(1))[0]

    def bool(self):
        return self.u8() != 0

    def i16(self):
        return struct.unpack(">h", self.take(2))[0]

    def u16(self):
        return struct.unpack(">H", self.take(2))[0]

    def i32(self):
        return struct.unpack(">i", self.take(4))[0]

    def i64(self):
        return struct.unpack(">q", self.take(8))[0]

    def f64(self):
        return struct.unpack(">d", self.take(8))[0]

    def utf(self):
        """DataInput.readUTF: u16 length, modified UTF-8"""
        return self.take(self.u16()).decode("utf-8", errors="surrogatepass")

    def peek(self):
        return self.b[self.pos]


class DataOutput:
    def __init__(self):
        self.buf = io.BytesIO()

    def write(self, b):
        self.buf.write(b)

    def u8(self, v):
        self.write(struct.pack(">B", v))

    def bool(self, v):
        self.u8(1 if v else 0)

    def i16(self, v):
        self.write(struct.pack(">h", v))

    def i32(self, v):
        self.write(struct.pack(">i", v))

    def i64(self, v):
        self.write(struct.pack(">q", v))

    def utf(self, s):
        b = s.encode("utf-8")
        self.write(struct.pack(">H", len(b)) + b)

    def getvalue(self):
        return self.buf.getvalue()


# ---------------------------------------------------------------- type serializers (data formats)
class LongSer:
    """LongSerializer: 8-byte big-endian"""

    def read(self, r):
        return r.i64()

    def write(self, w, v):
        w.i64(v)


class IntSer:
    def read(self, r):
        return r.i32()

    def write(self, w, v):
        w.i32(v)


class StringSer:
    """StringSerializer -> StringValue.writeString/readString (StringValue.java:745-830): length + 1 as a base-128
    varint (0 = null), then each UTF-16 char as a base-128 varint"""

    @staticmethod
    def _varint(r):
        v, shift = 0, 0
        while True:
            c = r.u8()
            v |= (c & 0x7F) << shift
            if c < 0x80:
                return v
            shift += 7

    @staticmethod
    def _put_varint(w, v):
        while v >= 0x80:
            w.u8((v & 0x7F) | 0x80)
            v >>= 7
        w.u8(v)

    def read(self, r):
        n = self._varint(r)
        if n == 0:
            return None
        units = [self._varint(r) for _ in range(n - 1)]
        return struct.pack(f"<{len(units)}H", *units).decode("utf-16-le", errors="surrogatepass")

    def write(self, w, s):
        if s is None:
            w.u8(0)
            return
        units = struct.unpack(f"<{len(s.encode('utf-16-le')) // 2}H", s.encode("utf-16-le", errors="surrogatepass"))
        self._put_varint(w, len(units) + 1)
        for u in units:
            self._put_varint(w, u)


class TimeWindowSer:
    """TimeWindow.Serializer: start, end (TimeWindow.java:147-208)"""

    def read(self, r):
        return (r.i64(), r.i64())

    def write(self, w, v):
        w.i64(v[0])
        w.i64(v[1])


class TupleSer:
    """TupleSerializer: the fields in order, no null mask"""

    def __init__(self, *fields):
        self.fields = fields

    def read(self, r):
        return tuple(f.read(r) for f in self.fields)

    def write(self, w, v):
        for f, x in zip(self.fields, v):
            f.write(w, x)


class ListSer:
    """ArrayListSerializer (flink-runtime/.../state/ArrayListSerializer.java:91-108): size, elements — the heap
    ListState's value"""

    def __init__(self, elem):
        self.elem = elem

    def read(self, r):
        return [self.elem.read(r) for _ in range(r.i32())]

    def write(self, w, v):
        w.i32(len(v))
        for x in v:
            self.elem.write(w, x)


class StreamRecordSer:
    """StreamElementSerializer of a StreamRecord (StreamElementSerializer.java:167-221): tag 0 + timestamp + value,
    or tag 1 + value (no timestamp: read back as timestamp None) — the EvictingWindowOperator's list elements"""

    def __init__(self, value):
        self.value = value

    def read(self, r):
        tag = r.u8()
        if tag == 0:
            ts = r.i64()
            return (ts, self.value.read(r))
        if tag == 1:
            return (None, self.value.read(r))
        raise ValueError(f"Corrupt stream, found tag: {tag}")

    def write(self, w, v):
        ts, val = v
        if ts is None:
            w.u8(1)
        else:
            w.u8(0)
            w.i64(ts)
        self.value.write(w, val)


# ---------------------------------------------------------------- Java serialization stream (skipped, not decoded)
_PRIM = {"B": 1, "C": 2, "D": 8, "F": 4, "I": 4, "J": 8, "S": 2, "Z": 1}
_BASE_HANDLE = 0x7E0000


class _Desc:
    def __init__(self, name):
        self.name, self.flags, self.fields, self.sup = name, 0, [], None


class JavaStreamSkipper:
    """Walks one object of the Java Object Serialization Stream Protocol (magic 0xACED, version 5) and returns the
    class name of the top-level object; nothing is instantiated."""

    def __init__(self, r):
        self.r = r
        self.handles = []

    def skip_stream(self):
        if self.r.u16() != 0xACED or self.r.u16() != 5:
            raise ValueError("not a Java serialization stream")
        return self._object()

    def _reg(self, obj):
        self.handles.append(obj)
        return obj

    def _object(self):
        r = self.r
        tc = r.u8()
        if tc == 0x70:  # TC_NULL
            return None
        if tc == 0x71:  # TC_REFERENCE
            return self.handles[r.i32() - _BASE_HANDLE]
        if tc == 0x72:  # TC_CLASSDESC
            return self._new_desc()
        if tc == 0x7D:  # TC_PROXYCLASSDESC
            d = self._reg(_Desc("<proxy>"))
            for _ in range(r.i32()):
                r.utf()
            self._annotation()
            d.sup = self._desc()
            return d
        if tc == 0x73:  # TC_OBJECT
            d = self._desc()
            self._reg(("object", d.name if d else None))
            self._classdata(d)
            return d.name if d else None
        if tc == 0x74:  # TC_STRING
            return self._reg(r.utf())
        if tc == 0x7C:  # TC_LONGSTRING
            return self._reg(r.take(r.i64()).decode("utf-8", errors="surrogatepass"))
        if tc == 0x75:  # TC_ARRAY
            d = self._desc()
            self._reg(("array", d.name))
            n = r.i32()
            comp = d.name[1]
            for _ in range(n):
                if comp in _PRIM:
                    r.take(_PRIM[comp])
                else:
                    self._object()
            return d.name
        if tc == 0x76:  # TC_CLASS
            d = self._desc()
            self._reg(("class", d.name if d else None))
            return d.name if d else None
        if tc == 0x7E:  # TC_ENUM
            d = self._desc()
            self._reg(("enum", d.name))
            self._object()
            return d.name
        if tc in (0x77, 0x7A):  # block data inside an annotation
            r.take(r.u8() if tc == 0x77 else r.i32())
            return None
        raise ValueError(f"unsupported Java serialization type code 0x{tc:02x} at {r.pos - 1}")

    def _desc(self):
        obj = self._object()
        if obj is not None and not isinstance(obj, _Desc):
            raise ValueError("expected a class descriptor")
        return obj

    def _new_desc(self):
        r = self.r
        d = self._reg(_Desc(r.utf()))
        r.i64()  # serialVersionUID
        d.flags = r.u8()
        for _ in range(r.i16()):
            code = chr(r.u8())
            r.utf()  # field name
            if code in "L[":
                self._object()  # the field's class name (a string or a reference)
            d.fields.append(code)
        self._annotation()
        d.sup = self._desc()
        return d

    def _annotation(self):
        while True:
            if self.r.peek() == 0x78:  # TC_ENDBLOCKDATA
                self.r.u8()
                return
            self._object()

    def _classdata(self, d):
        chain = []
        while d is not None:
            chain.append(d)
            d = d.sup
        for c in reversed(chain):
            if c.flags & 0x04:  # SC_EXTERNALIZABLE (block-data mode)
                self._annotation()
                continue
            if c.flags & 0x02:  # SC_SERIALIZABLE
                for code in c.fields:
                    if code in _PRIM:
                        self.r.take(_PRIM[code])
                    else:
                        self._object()
                if c.flags & 0x01:  # SC_WRITE_METHOD: writeObject's extra data
                    self._annotation()


def skip_resilient_serializers(r):
    """TypeSerializerSerializationUtil.readSerializersAndConfigsWithResilience: the count, the offset pairs, the total
    length and the block — skipped whole (:174-214); returns the block's bytes as written (the writers below put
    them back verbatim: the host owns its serializers, this module never builds one)"""
    start = r.pos
    n = r.i32()
    for _ in range(2 * n):
        r.i32()
    r.take(r.i32())
    return r.b[start:r.pos]


# ---------------------------------------------------------------- operator snapshot file
class KeyedHandle:
    """KeyGroupsStateHandle: key groups [start, start + len(offsets)) at `offsets` into `data`"""

    def __init__(self, start, offsets, name, data):
        self.start, self.offsets, self.name, self.data = start, offsets, name, data

    def key_groups(self):
        return range(self.start, self.start + len(self.offsets))


def _stream_handle(r):
    t = r.u8()
    if t == 0:
        return None
    if t == 1:  # ByteStreamStateHandle: name, data
        name = r.utf()
        return name, r.take(r.i32())
    if t == 2:
        raise ValueError("FileStateHandle: the state lives in a file outside the snapshot")
    raise ValueError(f"unknown stream state handle type {t}")


def _keyed_handle(r):
    t = r.u8()
    if t == 0:
        return None
    if t != 3:
        raise ValueError(f"unknown keyed state handle type {t}")
    start, n = r.i32(), r.i32()
    offsets = [r.i64() for _ in range(n)]
    h = _stream_handle(r)
    return KeyedHandle(start, offsets, h[0], h[1]) if h else None


def _operator_handle(r):
    t = r.u8()
    if t == 0:
        return None
    if t != 4:
        raise ValueError(f"unknown operator state handle type {t}")
    for _ in range(r.i32()):
        r.utf()
        r.u8()
        for _ in range(r.i32()):
            r.i64()
    _stream_handle(r)
    return t


def read_operator_snapshot(data):
    """OperatorSnapshotUtil.readStateHandle: {"raw_keyed": [KeyedHandle], "managed_keyed": [KeyedHandle], ...}"""
    r = DataInput(data)
    out = {"chain_index": r.i32()}
    _stream_handle(r)  # legacy state handle
    for kind, reader in (("raw_operator", _operator_handle), ("managed_operator", _operator_handle),
                         ("raw_keyed", _keyed_handle), ("managed_keyed", _keyed_handle)):
        n = r.i32()
        out[kind] = None if n < 0 else [reader(r) for _ in range(n)]
    if r.pos != len(r.b):
        raise ValueError("trailing bytes after the operator snapshot")
    return out


# ---------------------------------------------------------------- heap keyed state
STATE_TYPES = ["UNKNOWN", "VALUE", "LIST", "REDUCING", "FOLDING", "AGGREGATING", "MAP"]  # StateDescriptor.Type


def read_heap_keyed_state(handle, serializers):
    """The managed keyed state of a heap backend: ({"version", "compression", "states": [(type, name)]},
    {key group: {state name: [(namespace, key, value)]}}).  serializers[name] = (namespace, key, value) data
    serializers of that state."""
    r = DataInput(handle.data)
    version = r.i32()
    if version < 3:
        raise ValueError(f"serialization proxy version {version}: serializers without length prefixes (Flink 1.2)")
    compression = r.bool() if version >= 4 else False
    if compression:
        raise ValueError("snappy-compressed key groups are not read")
    blocks = {"key": skip_resilient_serializers(r)}  # the key serializer
    states = []
    for _ in range(r.i16()):
        typ = r.i32()
        name = r.utf()
        blocks[name] = skip_resilient_serializers(r)  # namespace and state serializers
        states.append((STATE_TYPES[typ] if 0 <= typ < len(STATE_TYPES) else typ, name))
    meta = {"version": version, "compression": compression, "states": states, "header_end": r.pos,
            "serializers": blocks}
    groups = {}
    for kg, off in zip(handle.key_groups(), handle.offsets):
        r.pos = off
        groups[kg] = read_key_group_section(r, kg, [n for _, n in states], serializers)
    return meta, groups


def read_key_group_section(r, kg, names, serializers):
    """one key group's section: {state name: [(namespace, key, value)]}; names = the states in id order"""
    if r.i32() != kg:
        raise ValueError(f"key group {kg}: section starts with another id")
    per = {}
    for _ in names:
        name = names[r.i16()]
        ns, key, val = serializers[name]
        per[name] = [(ns.read(r), key.read(r), val.read(r)) for _ in range(r.i32())]
    return per


def write_key_group_section(kg, states, serializers):
    """HeapKeyedStateBackend's key-group section (:375-381 + CopyOnWriteStateTableSnapshot.writeMappingsInKeyGroup):
    states = [(state id, name, [(namespace, key, value)])]"""
    w = DataOutput()
    w.i32(kg)
    for sid, name, mappings in states:
        ns, key, val = serializers[name]
        w.i16(sid)
        w.i32(len(mappings))
        for n, k, v in mappings:
            ns.write(w, n)
            key.write(w, k)
            val.write(w, v)
    return w.getvalue()


def write_keyed_state_stream(header, sections):
    """A keyed state stream: the serialization proxy bytes (`header`, as the backend's own writer produces them)
    followed by the key-group sections; returns (bytes, offsets)"""
    out, offsets = bytearray(header), []
    for sec in sections:
        offsets.append(len(out))
        out += sec
    return bytes(out), offsets


def write_serialization_proxy(version, key_serializer, states, compression=False):
    """KeyedBackendSerializationProxy.write (KeyedBackendSerializationProxy.java:101-118): the version (VersionedIO
    ReadableWritable: a bare int), the key-group compression flag from version 4 on, the key serializer block, then
    per registered state its type ordinal, name and namespace / state serializer block (the V3 meta-info writer,
    KeyedBackendStateMetaInfoSnapshotReaderWriters.java:96-116).  states = [(type name, state name, serializer
    block)]; the serializer blocks are the host's (TypeSerializerSerializationUtil.writeSerializersAndConfigsWith
    Resilience output, as read_heap_keyed_state returns them in meta["serializers"]).  Versions 3 and 4."""
    if version not in (3, 4):
        raise ValueError(f"serialization proxy version {version}: 3 (Flink 1.3) or 4 (1.4, 1.5) are written")
    if compression:
        raise ValueError("snappy-compressed key groups are not written")
    w = DataOutput()
    w.i32(version)
    if version >= 4:
        w.bool(False)
    w.write(bytes(key_serializer))
    w.i16(len(states))
    for typ, name, block in states:
        w.i32(STATE_TYPES.index(typ) if isinstance(typ, str) else int(typ))
        w.utf(name)
        w.write(bytes(block))
    return w.getvalue()


# ---------------------------------------------------------------- iteration orders of the heap backend
# A snapshot writes its mappings and timers in the order the JVM's hash structures iterate them, so equal state
# gives equal bytes only in that order.  These restate the orders from the structures' definitions.
def long_to_int_with_bit_mixing(v):
    """MathUtils.longToIntWithBitMixing (MathUtils.java:177-182)"""
    m = (1 << 64) - 1
    v &= m
    v = ((v ^ (v >> 30)) * 0xBF58476D1CE4E5B9) & m
    v = ((v ^ (v >> 27)) * 0x94D049BB133111EB) & m
    v ^= v >> 31
    return _i32(v)


def time_window_hash(w):
    """TimeWindow.hashCode (TimeWindow.java:102-104): longToIntWithBitMixing(start + end)"""
    return long_to_int_with_bit_mixing(w[0] + w[1])


def timer_hash(key_hash, ns_hash, ts):
    """InternalTimer.hashCode (InternalTimer.java:84-89)"""
    t = ts & ((1 << 64) - 1)
    h = _i32(t ^ (t >> 32))
    h = _i32(31 * h + key_hash)
    return _i32(31 * h + ns_hash)


def state_table_order(mappings, key_hash, ns_hash, capacity=1024):
    """The order CopyOnWriteStateTable's snapshot walks `mappings` [(namespace, key, state)] inserted in the given
    order: buckets in index order (compositeHash = bitMix(key.hashCode() ^ namespace.hashCode()) & (capacity - 1),
    CopyOnWriteStateTable.java:831-834; default capacity 1024, doubled past 3/4 load, :197-247 / :626-637), each
    bucket's chain newest first (addNewStateTableEntry puts the entry at the chain's head, :643-675).

    Exact for tables that never grew: putEntry doubles when size() > threshold BEFORE adding (:486-490), so m
    mappings stay at the initial capacity while m - 1 <= 3/4 of it (769 at 1024).  A table that grew is rehashed
    incrementally, MIN_TRANSFERRED_PER_INCREMENTAL_REHASH entries per later get or put (:735-780), each moved chain
    reversed into the new table, and a snapshot during the rehash walks both arrays (snapshotTableArrays, :599-614):
    its order depends on how many operations followed the doubling and on removals, which the mappings alone do not
    tell.  For such tables this returns a deterministic order at the grown capacity (newest first): the savepoint is
    valid and restores the same state, but is not byte-identical to the JVM's."""
    cap = capacity
    while len(mappings) - 1 > (cap >> 1) + (cap >> 2):
        cap <<= 1
    b = [bit_mix(key_hash(k) ^ ns_hash(n)) & (cap - 1) for n, k, _ in mappings]
    return [mappings[i] for i in sorted(range(len(mappings)), key=lambda i: (b[i], -i))]


def hash_set_order(items, hash_of):
    """The iteration order of a java.util.HashSet built by adding `items` in order to `new HashSet<>()` (initial
    capacity 16, load factor 0.75; the table doubles when the size exceeds 3/4 of it and a split keeps each bucket's
    relative order): buckets by (h ^ (h >>> 16)) & (capacity - 1), insertion order inside a bucket.  Buckets of 8 or
    more (tree bins) are not modelled."""
    cap = 16
    while len(items) > (cap * 3) // 4:
        cap <<= 1
    def bucket(x):
        h = hash_of(x) & 0xFFFFFFFF
        return (h ^ (h >> 16)) & (cap - 1)
    b = [bucket(x) for x in items]
    return [items[i] for i in sorted(range(len(items)), key=lambda i: (b[i], i))]


def nested_maps_order(mappings, key_hash, ns_hash):
    """The order NestedMapsStateTable's snapshot writes one key group's mappings (the heap backend's table with
    synchronous snapshots: a HashMap of namespaces, each a HashMap of keys, NestedMapsStateTable.java:221-238 and
    :352-368): namespaces in HashMap order, then each namespace's keys in HashMap order (first insertion = the
    given order)."""
    by_ns = {}
    for n, k, v in mappings:
        by_ns.setdefault(n, []).append((n, k, v))
    out = []
    for n in hash_set_order(list(by_ns), ns_hash):
        out += hash_set_order(by_ns[n], lambda m: key_hash(m[1]))
    return out


def heap_section_order(mappings, key_hash, ns_hash, table="copy_on_write"):
    """One key group's mappings in the order the heap backend's snapshot writes them: "copy_on_write"
    (CopyOnWriteStateTable, asynchronous snapshots: state_table_order, partitioned by key group without reordering,
    CopyOnWriteStateTableSnapshot.partitionEntriesByKeyGroup, CopyOnWriteStateTableSnapshot.java:127-167) or
    "nested_maps" (NestedMapsStateTable, synchronous snapshots: HeapKeyedStateBackend.newStateTable,
    HeapKeyedStateBackend.java:614-618)."""
    if table == "nested_maps":
        return nested_maps_order(list(mappings), key_hash, ns_hash)
    if table != "copy_on_write":
        raise ValueError(f"unknown heap state table {table!r}")
    return state_table_order(list(mappings), key_hash, ns_hash)


def timer_set_order(timers, key_hash, ns_hash):
    """hash_set_order of one key group's timers (HeapInternalTimerService keeps a HashSet per key group,
    HeapInternalTimerService.java:361-367)"""
    return hash_set_order(list(timers), lambda t: timer_hash(key_hash(t[0]), ns_hash(t[1]), t[2]))


# ---------------------------------------------------------------- KeyGroupsStateHandle / operator snapshot file
def write_keyed_handle(start, offsets, name, data):
    """SavepointV1Serializer.serializeKeyedStateHandle (SavepointV1Serializer.java:262-280): type 3 (key groups),
    the first key group, the offsets of the range's key groups, then the ByteStreamStateHandle (type 1: name, data)"""
    w = DataOutput()
    w.u8(3)
    w.i32(start)
    w.i32(len(offsets))
    for o in offsets:
        w.i64(o)
    w.u8(1)
    w.utf(name)
    w.i32(len(data))
    w.write(bytes(data))
    return w.getvalue()


def write_operator_snapshot(chain_index, raw_keyed, managed_keyed):
    """OperatorSnapshotUtil.writeStateHandle (OperatorSnapshotUtil.java:48-76): chain index, no legacy handle, no
    raw / managed operator state, then the raw and managed keyed handles (each a list of write_keyed_handle bytes;
    None = absent)"""
    w = DataOutput()
    w.i32(chain_index)
    w.u8(0)  # legacy operator state
    for handles in (None, None, raw_keyed, managed_keyed):
        if handles is None:
            w.i32(-1)
            continue
        w.i32(len(handles))
        for h in handles:
            w.write(h)
    return w.getvalue()


# ---------------------------------------------------------------- timers (raw keyed state)
_VERSIONED = bytes([0xF1, 0xCD, 0x85, 0x9F])  # PostVersionedIOReadableWritable.VERSIONED_IDENTIFIER


def read_timers(handle, key_ser, ns_ser, meta=None):
    """{key group: {service name: (event-time timers, processing-time timers)}}, a timer = (key, namespace, ts).
    meta (a dict, optional) receives per key group {"versioned": bool, "serializers": {service: bytes}}: the
    format of the section and each service's serializer bytes as written (write_timer_section puts them back)."""
    out = {}
    for kg, off in zip(handle.key_groups(), handle.offsets):
        r = DataInput(handle.data, off)
        versioned = r.b[off:off + 4] == _VERSIONED
        if versioned:
            r.take(4)
            r.i32()  # proxy version
        services, sers = {}, {}
        for _ in range(r.i32()):
            name = r.utf()
            s0 = r.pos
            if versioned:
                skip_resilient_serializers(r)
            else:  # pre-versioned: the key and namespace serializers as bare Java serialization streams
                JavaStreamSkipper(r).skip_stream()
                JavaStreamSkipper(r).skip_stream()
            sers[name] = r.b[s0:r.pos]
            ev = [(key_ser.read(r), ns_ser.read(r), r.i64()) for _ in range(r.i32())]
            pt = [(key_ser.read(r), ns_ser.read(r), r.i64()) for _ in range(r.i32())]
            services[name] = (ev, pt)
        out[kg] = services
        if meta is not None:
            meta[kg] = {"versioned": versioned, "serializers": sers}
    return out


def write_timer_section(services, key_ser, ns_ser, versioned=True):
    """One key group's raw keyed state: InternalTimeServiceManager.snapshotStateForKeyGroup (InternalTimeService
    Manager.java:114-118) -> InternalTimerServiceSerializationProxy.write (InternalTimerServiceSerializationProxy.java:
    92-106): the post-versioned identifier and proxy version 1, the number of timer services, then per service its
    name, the key / namespace serializers and the timers (InternalTimersSnapshotReaderWriters.java:96-160: event-time
    count + timers, processing-time count + timers; a timer = key, namespace, timestamp, InternalTimer.java:148-159).
    services = [(name, serializer bytes, event timers, processing timers)]; the serializer bytes are the host's:
    the resilient block (versioned) or two bare Java serialization streams (pre-versioned, Flink 1.4.0 and 1.3,
    versioned=False, which also drops the identifier).  Timers are written in the given order (timer_set_order
    gives the heap's)."""
    w = DataOutput()
    if versioned:
        w.write(_VERSIONED)
        w.i32(1)
    w.i32(len(services))
    for name, sers, ev, pt in services:
        w.utf(name)
        w.write(bytes(sers))
        for timers in (ev, pt):
            w.i32(len(timers))
            for k, n, ts in timers:
                key_ser.write(w, k)
                ns_ser.write(w, n)
                w.i64(ts)
    return w.getvalue()


def write_savepoint_key_group_0(meta, timer_meta, mappings, event_timers, serializers, chain_index, managed_name,
                                raw_name, table="copy_on_write", key_hash=None, ns_hash=None):
    """A WindowOperator's savepoint file for a one-key-group range (the test harness' maxParallelism 1: key group 0)
    from its content: `mappings` [(window, key, state)] of the one registered state and the `event_timers` of
    "window-timers" (any order: written in the heap's iteration order, `table` as in heap_section_order), with the
    host's serializer blocks and handle names (meta / timer_meta as read_heap_keyed_state / read_timers return
    them).  String keys and TimeWindow namespaces unless key_hash / ns_hash say otherwise."""
    from .keygroups import string_hash_code
    key_hash = key_hash or string_hash_code
    ns_hash = ns_hash or time_window_hash
    (typ, name), = meta["states"]
    hdr = write_serialization_proxy(meta["version"], meta["serializers"]["key"],
                                    [(typ, name, meta["serializers"][name])])
    sec = write_key_group_section(0, [(0, name, heap_section_order(mappings, key_hash, ns_hash, table))], serializers)
    stream, offsets = write_keyed_state_stream(hdr, [sec])
    timers = write_timer_section([("window-timers", timer_meta["serializers"]["window-timers"],
                                   timer_set_order(event_timers, key_hash, ns_hash), [])],
                                 serializers[name][1], serializers[name][0], versioned=timer_meta["versioned"])
    return write_operator_snapshot(chain_index, [write_keyed_handle(0, [0], raw_name, timers)],
                                   [write_keyed_handle(0, offsets, managed_name, stream)])


def rows_to_timers(rows, key_name, service_timer=lambda r: int(r["end"]) - 1):
    """the EventTimeTrigger timers (key, window, maxTimestamp) of GPU state rows whose `timer` is set"""
    return [(key_name(int(r["key"])), (int(r["start"]), int(r["end"])), service_timer(r)) for r in rows if r["timer"]]


# ---------------------------------------------------------------- heap state <-> GPU operator state
def event_timers(timers, service="window-timers"):
    """the set of (key, namespace, timestamp) event-time timers of one timer service over all key groups"""
    return {t for per in timers.values() for t in per.get(service, ([], []))[0]}


def reduce_rows_from_heap(mappings, timers, key_id, field, ordinal_base=0):
    """A ReducingState of sum(pos) / min(pos) / max(pos) over TimeWindows (the reduced element, HeapReducingState)
    as GPU state rows (fw_state_rows: key, start, end, count, sum, min, max = the element's ordinal, timer) plus the
    passthrough table {ordinal: element} the host keeps for the rows' other fields (FW_AGG_FIRST).  The heap state
    keeps no element count: restored rows count 1.  timer = the window's EventTimeTrigger timer (maxTimestamp) is
    among `timers`."""
    rows, passthrough = [], {}
    for i, ((start, end), key, elem) in enumerate(mappings):
        o = ordinal_base + i
        v = elem[field]
        rows.append(dict(key=key_id(key), start=start, end=end, count=1, sum=v, min=v, max=o,
                         timer=int((key, (start, end), end - 1) in timers)))
        passthrough[o] = elem
    return rows, passthrough


def heap_from_reduce_rows(rows, key_name, passthrough, field):
    """GPU state rows of a first-element reduce back to heap mappings: the passthrough element with the field
    replaced by the row's sum"""
    out = []
    for r in rows:
        e = list(passthrough[int(r["max"])])
        e[field] = int(r["sum"])
        out.append(((int(r["start"]), int(r["end"])), key_name(int(r["key"])), tuple(e)))
    return out


def trigger_counts_from_heap(count_mappings):
    """CountTrigger's partial counts: its ReducingState "count" (Sum over LongSerializer, CountTrigger.java:41-43,
    read with serializers (window, key, LongSer())) as {(key, window): count}"""
    return {(key, window): int(c) for window, key, c in count_mappings}


def list_state_from_heap(mappings, timers, key_id, value_of, ts_of=None, ordinal_base=0, trigger_counts=None):
    """A window-contents ListState (WindowOperator: the values; EvictingWindowOperator: StreamRecords) as the list
    operator's state: (lists [dict key, start, end, trigger_count, timer, n_elems], elements [(ts, val, ordinal)]).
    Values without a timestamp get Long.MIN_VALUE ("no timestamp").  trigger_counts: a CountTrigger's counts
    (trigger_counts_from_heap); without them every window restores with count 0, which is right only for
    EventTimeTrigger operators (the list operator refuses nothing here: the caller knows its trigger)."""
    lists, elems = [], []
    o = ordinal_base
    for (start, end), key, values in mappings:
        tc = trigger_counts.get((key, (start, end)), 0) if trigger_counts else 0
        lists.append(dict(key=key_id(key), start=start, end=end, trigger_count=tc,
                          timer=int((key, (start, end), end - 1) in timers), n_elems=len(values)))
        for v in values:
            ts = ts_of(v) if ts_of else None
            elems.append((-(1 << 63) if ts is None else ts, value_of(v), o))
            o += 1
    return lists, elems


def heap_from_list_state(lists, elems, key_name, make_value):
    """the list operator's state back to heap mappings [((start, end), key, [values])]"""
    out, k = [], 0
    for r in lists:
        n = int(r["n_elems"])
        out.append(((int(r["start"]), int(r["end"])), key_name(int(r["key"])),
                    [make_value(elems[k + j]) for j in range(n)]))
        k += n
    return out
