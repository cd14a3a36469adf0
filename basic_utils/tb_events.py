"""
Minimal TensorBoard event-file writer (scalars only), used when the
``tensorboard`` package is not installed (it is not, on the MI355X image).

Files are bit-compatible with TensorBoard's reader: TFRecord framing (u64
length, masked CRC32C of the length, payload, masked CRC32C of the payload)
around hand-encoded ``tensorflow.Event`` protobufs:

    Event   { double wall_time = 1; int64 step = 2; string file_version = 3;
              Summary summary = 5; }
    Summary { repeated Value value = 1; }
    Value   { string tag = 1; float simple_value = 2; }

Replaces the reference's TF1 ``EventsWriter`` path (reference:
basic_utils/logger.py:153-191; SURVEY O-5/C7).
"""
import os
import socket
import struct
import time

_CRC_TABLE = []


def _crc_table():
    if not _CRC_TABLE:
        poly = 0x82F63B78  # CRC-32C (Castagnoli), reflected
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ poly if c & 1 else c >> 1
            _CRC_TABLE.append(c)
    return _CRC_TABLE


def crc32c(data):
    t = _crc_table()
    c = 0xFFFFFFFF
    for b in data:
        c = t[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc(data):
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


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


def _field_bytes(num, payload):
    return _varint((num << 3) | 2) + _varint(len(payload)) + payload


def encode_event(wall_time, step=None, file_version=None, scalars=None):
    msg = bytearray(struct.pack("<Bd", (1 << 3) | 1, wall_time))
    if step is not None:
        msg += _varint((2 << 3) | 0) + _varint(int(step))
    if file_version is not None:
        msg += _field_bytes(3, file_version.encode())
    if scalars:
        summary = bytearray()
        for tag, val in scalars.items():
            value = _field_bytes(1, str(tag).encode()) + struct.pack("<Bf", (2 << 3) | 5, float(val))
            summary += _field_bytes(1, value)
        msg += _field_bytes(5, bytes(summary))
    return bytes(msg)


def frame(record):
    header = struct.pack("<Q", len(record))
    return header + struct.pack("<I", masked_crc(header)) + record + struct.pack("<I", masked_crc(record))


class EventFileWriter:
    def __init__(self, logdir):
        os.makedirs(logdir, exist_ok=True)
        name = "events.out.tfevents.%010d.%s" % (int(time.time()), socket.gethostname())
        self.path = os.path.join(logdir, name)
        self._f = open(self.path, "ab")
        self._f.write(frame(encode_event(time.time(), file_version="brain.Event:2")))
        self._f.flush()

    def add_scalars(self, scalars, step):
        self._f.write(frame(encode_event(time.time(), step=step, scalars=scalars)))
        self._f.flush()

    def close(self):
        if self._f is not None:
            self._f.close()
            self._f = None


# ---- reader (tests / tooling) -----------------------------------------------------
def _read_varint(buf, i):
    shift = n = 0
    while True:
        b = buf[i]
        i += 1
        n |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            return n, i


def _fields(buf):
    i = 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(buf, i)
        elif wt == 1:
            v = struct.unpack_from("<d", buf, i)[0]
            i += 8
        elif wt == 5:
            v = struct.unpack_from("<f", buf, i)[0]
            i += 4
        elif wt == 2:
            ln, i = _read_varint(buf, i)
            v = bytes(buf[i:i + ln])
            i += ln
        else:
            raise ValueError("unsupported wire type %d" % wt)
        yield num, v


def read_events(path):
    """-> list of (step, {tag: value}); verifies every CRC."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        header = data[i:i + 8]
        (ln,) = struct.unpack("<Q", header)
        assert struct.unpack_from("<I", data, i + 8)[0] == masked_crc(header), "header crc"
        rec = data[i + 12:i + 12 + ln]
        assert struct.unpack_from("<I", data, i + 12 + ln)[0] == masked_crc(rec), "record crc"
        i += 16 + ln
        step, scalars = None, {}
        for num, v in _fields(rec):
            if num == 2:
                step = v
            elif num == 5:
                for _, val in _fields(v):
                    tag, sv = None, None
                    for n2, v2 in _fields(val):
                        if n2 == 1:
                            tag = v2.decode()
                        elif n2 == 2:
                            sv = v2
                    scalars[tag] = sv
        if scalars:
            out.append((step, scalars))
    return out
