"""TFRecord files and tf.train.Example records without TensorFlow.

Formats (public TensorFlow specs):
  TFRecord frame : uint64 length | uint32 masked_crc32c(length) | data | uint32 masked_crc32c(data)
  masked crc     : ((crc >> 15) | (crc << 17)) + 0xa282ead8  (mod 2^32), crc = CRC-32C (Castagnoli)
  Example        : 1: Features ; Features: 1: repeated map entry {1: key string, 2: Feature}
  Feature        : oneof 1: BytesList, 2: FloatList, 3: Int64List ; *List: 1: repeated value
                   (float/int64 packed when written by TF; unpacked is accepted on read)
The reader is what utils/data_loader.py's TFRecordDataset + parse_single_example
(reference utils/data_loader.py:7-30) does for the FixedLenFeature spec.
"""
import struct

import numpy as np

_POLY = 0x82F63B78


def _make_table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ _POLY if c & 1 else c >> 1
        t.append(c)
    return t


_TABLE = _make_table()


def crc32c(data, crc=0):
    c = crc ^ 0xFFFFFFFF
    tab = _TABLE
    for b in data:
        c = tab[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc(data):
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ----------------------------------------------------------------- protobuf wire
def _varint(n):
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf, pos):
    shift = 0
    result = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _field(num, wire, payload):
    return _varint((num << 3) | wire) + payload


def _len_field(num, data):
    return _field(num, 2, _varint(len(data)) + data)


def encode_example(features):
    """features: dict name -> ('int64'|'float'|'bytes', sequence)."""
    entries = b""
    for name in sorted(features):
        kind, values = features[name]
        if kind == "int64":
            packed = b"".join(_varint(int(v)) for v in values)
            feat = _len_field(3, _len_field(1, packed))
        elif kind == "float":
            packed = np.asarray(values, dtype="<f4").tobytes()
            feat = _len_field(2, _len_field(1, packed))
        elif kind == "bytes":
            feat = _len_field(1, b"".join(_len_field(1, bytes(v)) for v in values))
        else:
            raise ValueError(kind)
        entry = _len_field(1, name.encode()) + _len_field(2, feat)
        entries += _len_field(1, entry)
    return _len_field(1, entries)


def _parse_list(buf, kind):
    pos, end = 0, len(buf)
    vals = []
    while pos < end:
        tag, pos = _read_varint(buf, pos)
        num, wire = tag >> 3, tag & 7
        if wire == 2:
            ln, pos = _read_varint(buf, pos)
            chunk = buf[pos:pos + ln]
            pos += ln
            if kind == "bytes":
                vals.append(bytes(chunk))
            elif kind == "float":
                vals.extend(np.frombuffer(bytes(chunk), dtype="<f4").tolist())
            else:
                p = 0
                while p < len(chunk):
                    v, p = _read_varint(chunk, p)
                    vals.append(v - (1 << 64) if v >= 1 << 63 else v)
        elif wire == 5:      # unpacked float
            vals.append(struct.unpack("<f", bytes(buf[pos:pos + 4]))[0])
            pos += 4
        elif wire == 0:      # unpacked int64
            v, pos = _read_varint(buf, pos)
            vals.append(v - (1 << 64) if v >= 1 << 63 else v)
        else:
            raise ValueError("unexpected wire type %d" % wire)
    return vals


def decode_example(data):
    """Returns dict name -> (kind, list of values)."""
    buf = memoryview(data)
    out = {}

    def fields(b):
        pos = 0
        while pos < len(b):
            tag, pos = _read_varint(b, pos)
            wire = tag & 7
            if wire != 2:
                raise ValueError("unexpected wire type %d" % wire)
            ln, pos = _read_varint(b, pos)
            yield tag >> 3, b[pos:pos + ln]
            pos += ln

    for num, feats in fields(buf):
        if num != 1:
            continue
        for num2, entry in fields(feats):
            if num2 != 1:
                continue
            key, feat = None, None
            for n3, v in fields(entry):
                if n3 == 1:
                    key = bytes(v).decode()
                elif n3 == 2:
                    feat = v
            kind, vals = "bytes", []
            if feat is not None:
                for n4, lst in fields(feat):
                    kind = {1: "bytes", 2: "float", 3: "int64"}[n4]
                    vals = _parse_list(lst, kind)
            out[key] = (kind, vals)
    return out


# ----------------------------------------------------------------- files
def write_records(path, records):
    with open(path, "wb") as f:
        for data in records:
            ln = struct.pack("<Q", len(data))
            f.write(ln)
            f.write(struct.pack("<I", masked_crc(ln)))
            f.write(data)
            f.write(struct.pack("<I", masked_crc(data)))


def read_records(path, check_crc=True):
    with open(path, "rb") as f:
        while True:
            head = f.read(12)
            if not head:
                return
            if len(head) < 12:
                raise IOError("truncated record header in %s" % path)
            ln = struct.unpack("<Q", head[:8])[0]
            if check_crc and struct.unpack("<I", head[8:])[0] != masked_crc(head[:8]):
                raise IOError("corrupted record length in %s" % path)
            data = f.read(ln)
            crc = f.read(4)
            if len(data) < ln or len(crc) < 4:
                raise IOError("truncated record in %s" % path)
            if check_crc and struct.unpack("<I", crc)[0] != masked_crc(data):
                raise IOError("corrupted record data in %s" % path)
            yield data
