"""Zarr v2 source/sink format and chunk codecs, on CPU.

The reference writes Zarr v2 stores through zarr + numcodecs (absent here:
parity with numcodecs' own output is unpinned).  These tests pin the native
codec (cubed_amd/csrc/codec.cpp) against the published formats instead:

* Blosc 1.x frames assembled here byte by byte from the format description
  (header, block starts, split streams, byte shuffle, memcpyed and leftover
  blocks), with lz4 and zlib streams -- the decoder must read them all;
* every frame the encoder writes is re-decoded by an independent pure-Python
  LZ4 block decoder written from the LZ4 block-format spec (test only);
* Zarr v2 directory stores: metadata keys/encodings, chunk naming, full-shape
  edge chunks, fill values for missing chunks, codecs none/zlib/gzip/blosc,
  C and F order."""

import json
import os
import struct
import zlib

import numpy as np
import pytest

from cubed_amd import zarr_io as Z

# ----------------------------------------------------------------- helpers


def py_lz4_decode(src: bytes, size: int) -> bytes:
    """LZ4 block decoder from the format spec (test oracle)."""
    out = bytearray()
    i = 0
    while i < len(src):
        tok = src[i]
        i += 1
        lit = tok >> 4
        if lit == 15:
            while True:
                b = src[i]
                i += 1
                lit += b
                if b != 255:
                    break
        out += src[i:i + lit]
        i += lit
        if i >= len(src):
            break
        off = src[i] | src[i + 1] << 8
        i += 2
        ml = tok & 15
        if ml == 15:
            while True:
                b = src[i]
                i += 1
                ml += b
                if b != 255:
                    break
        ml += 4
        assert 0 < off <= len(out)
        for _ in range(ml):
            out.append(out[-off])
    assert len(out) == size
    return bytes(out)


def py_blosc_decode(frame: bytes) -> bytes:
    """Blosc 1.x frame reader over py_lz4_decode (test oracle for the encoder)."""
    ver, verlz, flags, ts = frame[0], frame[1], frame[2], frame[3]
    nbytes, bsize, cbytes = struct.unpack("<iii", frame[4:16])
    assert cbytes == len(frame)
    if flags & 2:
        return frame[16:16 + nbytes]
    assert flags >> 5 == 1
    nblocks = -(-nbytes // bsize)
    starts = struct.unpack(f"<{nblocks}i", frame[16:16 + 4 * nblocks])
    out = bytearray()
    for b, st in enumerate(starts):
        n = min(bsize, nbytes - b * bsize)
        leftover = n != bsize
        split = not (flags & 0x10) and not leftover and ts <= 16 and bsize // ts >= 128
        ns = ts if split else 1
        blk = bytearray()
        for _ in range(ns):
            cs = struct.unpack("<i", frame[st:st + 4])[0]
            st += 4
            data = frame[st:st + cs]
            st += cs
            blk += data if cs == n // ns else py_lz4_decode(data, n // ns)
        if flags & 1 and ts > 1:
            rows = n // ts
            a = np.frombuffer(bytes(blk[:rows * ts]), np.uint8).reshape(ts, rows).T.reshape(-1)
            blk = bytearray(a.tobytes()) + blk[rows * ts:]
        out += blk
    return bytes(out)


def lz4_literals(data: bytes) -> bytes:
    """An LZ4 block holding ``data`` as one literal run."""
    n = len(data)
    out = bytearray([min(n, 15) << 4])
    if n >= 15:
        r = n - 15
        while r >= 255:
            out.append(255)
            r -= 255
        out.append(r)
    return bytes(out) + data


def shuffle(block: bytes, ts: int) -> bytes:
    rows = len(block) // ts
    a = np.frombuffer(block[:rows * ts], np.uint8).reshape(rows, ts).T.reshape(-1)
    return a.tobytes() + block[rows * ts:]


def frame(data: bytes, ts: int, bsize: int, codec: int, do_shuffle: bool, dont_split: bool,
          encode) -> bytes:
    """Assemble a Blosc 1.x frame from the published layout."""
    nbytes = len(data)
    nblocks = -(-nbytes // bsize)
    flags = (codec << 5) | (1 if do_shuffle else 0) | (0x10 if dont_split else 0)
    body = bytearray()
    starts = []
    base = 16 + 4 * nblocks
    for b in range(nblocks):
        blk = data[b * bsize:(b + 1) * bsize]
        leftover = len(blk) != bsize
        if do_shuffle and ts > 1:
            blk = shuffle(blk, ts)
        split = not dont_split and not leftover and ts <= 16 and bsize // ts >= 128
        ns = ts if split else 1
        starts.append(base + len(body))
        ne = len(blk) // ns
        for j in range(ns):
            s = blk[j * ne:(j + 1) * ne]
            c = encode(s)
            if len(c) >= len(s):
                c = s
            body += struct.pack("<i", len(c)) + c
    hdr = bytes([2, 1, flags, ts]) + struct.pack("<iii", nbytes, bsize, base + len(body))
    return hdr + struct.pack(f"<{nblocks}i", *starts) + bytes(body)


def native_decode(fr: bytes, n: int) -> bytes:
    out = np.empty(n, np.uint8)
    Z._blosc_decompress(fr, out)
    return out.tobytes()


def patterned(n, seed=0):
    rng = np.random.default_rng(seed)
    # compressible: slowly varying floats with repeats
    return np.resize(np.repeat(rng.random(max(1, n // 64)), 64), n).astype(np.float32).tobytes()


# ----------------------------------------------------------------- blosc decoder vs spec frames


@pytest.mark.parametrize("ts, bsize, shuf, dont_split", [
    (4, 4096, True, False),    # split into 4 streams per block
    (4, 4096, True, True),     # unsplit
    (8, 2048, False, False),   # split, no shuffle
    (4, 256, True, False),     # blocksize/typesize = 64 < 128: never split
    (1, 1000, True, False),    # typesize 1: shuffle is a no-op
])
@pytest.mark.parametrize("codec", [1, 3])
def test_decoder_reads_spec_frames(built, ts, bsize, shuf, dont_split, codec):
    data = patterned(4 * 2500 + 3)  # leftover block and a typesize remainder
    enc = lz4_literals if codec == 1 else (lambda s: zlib.compress(s, 5))
    fr = frame(data, ts, bsize, codec, shuf, dont_split, enc)
    assert native_decode(fr, len(data)) == data


def test_decoder_lz4_matches_and_overlaps(built):
    # hand-written LZ4 sequences: a literal run, a far match, an overlapping
    # run-length match (offset 1) and a long match with extra length bytes
    lit = b"abcdefgh"
    seq = bytes([0x84]) + lit + struct.pack("<H", 8)                 # 8 literals, match 8 at -8
    seq += bytes([0x1F]) + b"z" + struct.pack("<H", 1) + bytes([255, 10])  # 1 literal, match 4+15+265 at -1
    seq += bytes([0x50]) + b"tail!"                                  # last literals
    expect = lit + lit + b"z" * (1 + 4 + 15 + 255 + 10) + b"tail!"
    data = expect
    fr = bytes([2, 1, (1 << 5) | 0x10, 1]) + struct.pack("<iii", len(data), len(data), 20 + 4 + len(seq))
    fr += struct.pack("<i", 20) + struct.pack("<i", len(seq)) + seq
    assert native_decode(fr, len(data)) == data
    assert py_lz4_decode(seq, len(data)) == data


def test_decoder_memcpyed_and_errors(built):
    data = bytes(range(200))
    fr = bytes([2, 1, 0x02 | (1 << 5), 1]) + struct.pack("<iii", 200, 200, 216) + data
    assert native_decode(fr, 200) == data
    with pytest.raises(ValueError):
        native_decode(fr, 100)  # size mismatch
    good = frame(patterned(8192), 4, 4096, 1, True, True, lz4_literals)
    bad = bytearray(good)
    bad[24:28] = struct.pack("<i", 1 << 30)  # first stream's size runs past the frame
    with pytest.raises(ValueError):
        native_decode(bytes(bad), 8192)
    bad = bytearray(good)
    bad[29] = 0  # literal run shorter than the block: the block decodes short
    with pytest.raises(ValueError):
        native_decode(bytes(bad), 8192)
    bitshuffled = bytes([2, 1, 0x04 | (1 << 5), 4]) + struct.pack("<iii", 8, 8, 40) + bytes(24)
    with pytest.raises(ValueError, match="unsupported"):
        native_decode(bitshuffled, 8)


# ----------------------------------------------------------------- encoder


@pytest.mark.parametrize("n", [0, 1, 5, 13, 127, 128, 4096, 300_001, 1 << 20])
@pytest.mark.parametrize("kind", ["pattern", "random", "zeros"])
def test_encoder_roundtrip_and_spec_decode(built, n, kind):
    if kind == "pattern":
        data = patterned(n // 4 + 1)[:n]
    elif kind == "random":
        data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    else:
        data = bytes(n)
    for ts, shuf in ((4, 1), (8, 1), (1, 0), (3, 1)):
        fr = Z._blosc_compress(np.frombuffer(data, np.uint8), ts, shuf)
        assert native_decode(fr, n) == data
        assert py_blosc_decode(fr) == data
    if kind != "random" and n >= 4096:
        assert len(fr) < n // 4  # it does compress


# ----------------------------------------------------------------- Zarr v2 stores


@pytest.mark.parametrize("compressor", ["default", None, {"id": "zlib", "level": 1},
                                        {"id": "gzip", "level": 5}])
@pytest.mark.parametrize("order, sep", [("C", "."), ("F", "/")])
def test_zarr_roundtrip(tmp_path, built, compressor, order, sep):
    x = np.random.default_rng(1).random((23, 17, 5))
    a = Z.ZarrV2Array.create(str(tmp_path / "a.zarr"), x.shape, x.dtype, (10, 8, 5), fill_value=-1.5,
                             compressor=compressor, order=order, dimension_separator=sep)
    a[...] = x
    b = Z.open_array(str(tmp_path / "a.zarr"))
    assert b.shape == x.shape and b.chunks == (10, 8, 5) and b.dtype == x.dtype
    assert np.array_equal(b[...], x)
    names = sorted(os.path.relpath(os.path.join(r, f), tmp_path / "a.zarr")
                   for r, _, fs in os.walk(tmp_path / "a.zarr") for f in fs if f != ".zarray")
    exp = sorted(os.path.join(*(f"{i}{sep}{j}{sep}0".split("/"))) for i in range(3) for j in range(3))
    assert names == exp
    # every stored chunk has the full chunk shape (edge chunks padded with the fill)
    full = np.empty((10, 8, 5))
    b.decode_into((2, 2, 0), full)
    assert np.all(full[3:] == -1.5) and np.all(full[:, 1:] == -1.5)
    assert np.array_equal(full[:3, :1], x[20:, 16:])


def test_zarr_metadata_and_missing_chunks(tmp_path, built):
    a = Z.open_array(str(tmp_path / "m.zarr"), mode="w", shape=(5, 4), dtype="f4", chunks=(2, 2),
                     fill_value=float("nan"))
    meta = json.load(open(tmp_path / "m.zarr" / ".zarray"))
    assert meta == {"zarr_format": 2, "shape": [5, 4], "chunks": [2, 2], "dtype": "<f4",
                    "compressor": {"id": "blosc", "cname": "lz4", "clevel": 5, "shuffle": 1, "blocksize": 0},
                    "fill_value": "NaN", "order": "C", "filters": None, "dimension_separator": "."}
    a.write_chunk((1, 1), np.ones((2, 2), np.float32))
    got = Z.open_array(str(tmp_path / "m.zarr"))[...]
    assert np.isnan(got[:2]).all() and np.array_equal(got[2:4, 2:], np.ones((2, 2)))
    with pytest.raises(FileExistsError):
        Z.open_array(str(tmp_path / "m.zarr"), mode="w-", shape=(5, 4), dtype="f4")
    with pytest.raises(FileNotFoundError):
        Z.open_array(str(tmp_path / "nope.zarr"))
    i = Z.open_array(str(tmp_path / "i.zarr"), mode="w", shape=(7,), dtype=np.int64, chunks=(3,), fill_value=7)
    assert json.load(open(tmp_path / "i.zarr" / ".zarray"))["dtype"] == "<i8"
    assert np.array_equal(i[...], np.full(7, 7))
    s = Z.open_array(str(tmp_path / "s.zarr"), mode="w", shape=(), dtype=np.float64, chunks=())
    s[...] = 3.25
    assert os.path.exists(tmp_path / "s.zarr" / "0") and s[...] == 3.25


def test_zarr_refuses_what_it_cannot_decode(tmp_path, built):
    os.makedirs(tmp_path / "q.zarr")
    meta = {"zarr_format": 2, "shape": [4], "chunks": [4], "dtype": "<f8", "fill_value": 0.0,
            "order": "C", "filters": None, "compressor": {"id": "snappy"}}
    json.dump(meta, open(tmp_path / "q.zarr" / ".zarray", "w"))
    with pytest.raises(NotImplementedError, match="snappy"):
        Z.open_array(str(tmp_path / "q.zarr"))
    # blosclz streams inside a blosc frame: refused with a clear error
    data = patterned(4096)
    fr = bytearray(frame(data, 4, 4096, 3, True, True, lambda b: zlib.compress(b, 5)))
    fr[2] = (fr[2] & 0x1F) | (0 << 5)  # codec 0 = blosclz (the streams are compressed)
    with pytest.raises(ValueError, match="blosclz"):
        native_decode(bytes(fr), len(data))


def _zstd():
    import ctypes

    try:
        z = ctypes.CDLL("libzstd.so.1")
    except OSError:
        pytest.skip("libzstd.so.1 not available")
    z.ZSTD_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    z.ZSTD_compress.restype = ctypes.c_size_t
    z.ZSTD_compressBound.argtypes = [ctypes.c_size_t]
    z.ZSTD_compressBound.restype = ctypes.c_size_t

    def compress(b: bytes, level=3) -> bytes:
        cap = z.ZSTD_compressBound(len(b))
        out = ctypes.create_string_buffer(cap)
        n = z.ZSTD_compress(out, cap, b, len(b), level)
        assert n < cap
        return out.raw[:n]
    return compress


@pytest.mark.parametrize("ts, bsize, shuf, dont_split", [(4, 4096, True, False), (8, 2048, False, True)])
def test_decoder_reads_zstd_blosc_frames(built, ts, bsize, shuf, dont_split):
    """Blosc(cname="zstd"): codec 4 streams, decoded by the system libzstd
    (zstd frames here are written by the same library's ZSTD_compress)."""
    zc = _zstd()
    data = patterned(4 * 2500 + 3)
    fr = frame(data, ts, bsize, 4, shuf, dont_split, zc)
    assert native_decode(fr, len(data)) == data


def test_zarr_reads_zstd_lz4_lzma_bz2_chunks(tmp_path, built):
    """Standalone numcodecs compressors: "zstd" (one zstd frame), "lz4" (int32
    size + one LZ4 block), "lzma" and "bz2" (Python's codecs)."""
    import bz2
    import lzma

    zc = _zstd()
    x = np.arange(24, dtype=np.float64).reshape(4, 6) * 1.5
    encs = {"zstd": zc, "lz4": lambda b: struct.pack("<i", len(b)) + lz4_literals(b),
            "lzma": lzma.compress, "bz2": bz2.compress}
    for cid, enc in encs.items():
        d = tmp_path / f"{cid}.zarr"
        os.makedirs(d)
        meta = {"zarr_format": 2, "shape": [4, 6], "chunks": [2, 3], "dtype": "<f8", "fill_value": 0.0,
                "order": "C", "filters": None, "compressor": {"id": cid}}
        json.dump(meta, open(d / ".zarray", "w"))
        for i in range(2):
            for j in range(2):
                blk = np.ascontiguousarray(x[2 * i:2 * i + 2, 3 * j:3 * j + 3])
                open(d / f"{i}.{j}", "wb").write(enc(blk.tobytes()))
        a = Z.open_array(str(d))
        assert np.array_equal(a[...], x), cid
        with pytest.raises(NotImplementedError, match="writing"):
            Z.ZarrV2Array.create(str(tmp_path / f"w{cid}.zarr"), (4,), np.float64, (2,), compressor={"id": cid})


def test_zarr_overwrite_removes_nested_chunks(tmp_path, built):
    """mode='w' over a '/'-separated array: chunks in nested directories go
    too, so a chunk the new write never touches reads back as fill_value."""
    p = str(tmp_path / "n.zarr")
    a = Z.ZarrV2Array.create(p, (4, 4), np.float64, (2, 2), fill_value=0.0, dimension_separator="/")
    a[...] = np.arange(16.0).reshape(4, 4)
    assert os.path.isdir(os.path.join(p, "1"))
    b = Z.ZarrV2Array.create(p, (4, 4), np.float64, (2, 2), fill_value=-2.0, mode="w",
                             dimension_separator="/")
    assert sorted(os.listdir(p)) == [".zarray"]
    b.write_chunk((0, 0), np.ones((2, 2)))
    got = Z.open_array(p)[...]
    assert np.array_equal(got[:2, :2], np.ones((2, 2))) and np.all(got[2:] == -2.0) and np.all(got[:, 2:] == -2.0)
