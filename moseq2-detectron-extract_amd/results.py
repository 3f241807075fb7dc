"""Result writers: the extraction h5 layout and the
keypoints TSV, fed by the writer data dict GPUExtractor.process_chunk returns.

=============================  =============================================
this module                    reference (M/ = moseq2_detectron_extract/)
=============================  =============================================
create_extract_h5              M/io/result.py:14-103
write_extracted_chunk_to_h5    M/io/result.py:106-130
dict_to_h5                     M/io/util.py:136-176
KeypointsTSVWriter             ResultWriterStep.__process_csv
                               M/pipeline/write_results_step.py:54-73
open_results                   ResultWriterStep.__init_h5 :34-39
=============================  =============================================

h5py is not installed in this image's interpreter, so ``open_results`` falls
back to ``MemoryH5``: the same dataset tree (names, shapes, dtypes,
descriptions) held in numpy arrays and saved as one ``.npz`` (dataset path ->
array) on close; with h5py present it opens a real ``results_XX.h5``.  The
TSV is appended chunk by chunk (the reference rewrites the whole table after
every chunk: O(n^2) in the session length); the file bytes are the same.
"""
from __future__ import annotations

import functools
import io
import os
import struct
import zlib
from typing import Dict, Optional

import numpy as np

from .features import keypoint_attributes, scalar_attributes

PACKAGE_VERSION = "moseq2-detectron-extract-amd v0.1"


class MemoryDataset:
    """numpy-backed stand-in for h5py.Dataset (assignment casts like h5py)."""

    def __init__(self, data: np.ndarray):
        self.data = data
        self.attrs: Dict[str, object] = {}

    @property
    def shape(self):
        return self.data.shape

    @property
    def dtype(self):
        return self.data.dtype

    def __getitem__(self, idx):
        return self.data[idx]

    def __setitem__(self, idx, value):
        self.data[idx] = np.asarray(value).astype(self.data.dtype)


class MemoryH5:
    """Minimal h5py.File stand-in: a flat tree of datasets keyed by path.

    The datasets named in `stream` (the crop stacks: 12.8 KB per frame, the
    bulk of the file) are deflated while the session runs: rows_written(rows)
    compresses each piece of their streams that the rows complete, so close()
    only finishes their streams and compresses the small datasets."""

    def __init__(self, path: Optional[str] = None, stream=("frames", "frames_mask"), level: int = 4):
        self.path = path
        self.datasets: Dict[str, MemoryDataset] = {}
        self.level = level
        self._stream_keys = tuple(stream) if path else ()
        self._streams: Dict[str, "_DeflateStream"] = {}
        self._filled = None  # per-row "written" flags of the streamed datasets
        self._pool = None

    @staticmethod
    def _key(name: str) -> str:
        return name.strip("/")

    def create_dataset(self, name, shape=None, dtype=None, data=None, compression=None, **kw):
        key = self._key(name)
        if key in self.datasets:
            raise ValueError(f"dataset {key} exists")
        if data is not None:
            arr = np.array(data, dtype=dtype) if dtype is not None else np.array(data)
            if shape is not None:
                arr = arr.reshape(shape)
        else:
            arr = np.zeros(() if shape is None else shape, dtype=dtype or "float32")
        ds = MemoryDataset(arr)
        self.datasets[key] = ds
        return ds

    def __setitem__(self, name, value):
        self.create_dataset(name, data=value)

    def __getitem__(self, name) -> MemoryDataset:
        return self.datasets[self._key(name)]

    def __contains__(self, name) -> bool:
        return self._key(name) in self.datasets

    def rows_written(self, rows) -> None:
        """Rows `rows` of the streamed datasets hold their final values:
        deflate every piece of their streams now complete (wherever it lies:
        a sharded session's rounds fill the frame range in several places)."""
        keys = [k for k in self._stream_keys if k in self.datasets and self.datasets[k].data.ndim >= 1]
        if not keys:
            return
        n = self.datasets[keys[0]].data.shape[0]
        if self._filled is None:
            self._filled = np.zeros(n, bool)
        rows = np.asarray(rows)
        if rows.size == 0:
            return
        self._filled[rows] = True
        for k in keys:
            self._stream(k).feed_rows(self._filled, int(rows.min()), int(rows.max()) + 1)

    def _stream(self, key):
        if key not in self._streams:
            if self._pool is None:
                import concurrent.futures as cf
                self._pool = cf.ThreadPoolExecutor(max(1, min(16, len(os.sched_getaffinity(0)))))
            self._streams[key] = _DeflateStream(self.datasets[key].data, self.level, self._pool)
        return self._streams[key]

    def close(self):
        if self.path:
            try:
                pre = {k: self._stream(k).finish() for k in self._stream_keys if k in self._streams}
                save_npz(self.path, {k: v.data for k, v in self.datasets.items()}, level=self.level,
                         precompressed=pre, pool=self._pool)
            finally:
                if self._pool is not None:
                    self._pool.shutdown()
                    self._pool = None
            self.path = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


_PIECE = 1 << 20  # bytes per independently deflated piece (a chunk's crop rows spread over the pool)
_ZIP64_AT = 0xFFFFFFFF  # sizes / offsets from which a member needs zip64 records (tests lower it)


def _deflate_pieces(data: memoryview, level: int, pool, final: bool = True) -> list:
    """Raw deflate of `data` as one stream made of independently compressed
    pieces (every piece but the last ends on a sync flush, the last one
    finishes the stream unless final=False -- pigz's layout), compressed in
    parallel: zlib releases the GIL while it works."""
    cuts = list(range(0, len(data), _PIECE)) or [0]
    last = len(cuts) - 1
    return list(pool.map(lambda i: _deflate_one(data[cuts[i]:cuts[i] + _PIECE], level, final and i == last),
                         range(len(cuts))))


def _deflate_one(piece, level: int, final: bool) -> bytes:
    """One independently deflated piece, ending on a sync flush unless it
    finishes the stream."""
    c = zlib.compressobj(level, zlib.DEFLATED, -15)
    return c.compress(piece) + c.flush(zlib.Z_FINISH if final else zlib.Z_SYNC_FLUSH)


def _npy_header(a: np.ndarray) -> bytes:
    hdr = io.BytesIO()
    np.lib.format.write_array_header_1_0(hdr, np.lib.format.header_data_from_array_1_0(a))
    return hdr.getvalue()


def _gf2_times(mat, vec: int) -> int:
    s, i = 0, 0
    while vec:
        if vec & 1:
            s ^= mat[i]
        vec >>= 1
        i += 1
    return s


@functools.lru_cache(maxsize=8)
def _crc_zeros_op(nbytes: int) -> tuple:
    """The GF(2) operator (32 columns) that advances a CRC-32 over `nbytes`
    zero bytes: crc(A || B) = op(len B)(crc(A)) ^ crc(B) (zlib's
    crc32_combine, restated)."""
    op = [1 << n for n in range(32)]  # identity
    sq = [0xEDB88320] + [1 << n for n in range(31)]  # one zero bit
    for _ in range(3):  # -> one zero byte
        sq = [_gf2_times(sq, sq[n]) for n in range(32)]
    while nbytes:
        if nbytes & 1:
            op = [_gf2_times(sq, op[n]) for n in range(32)]
        nbytes >>= 1
        if nbytes:
            sq = [_gf2_times(sq, sq[n]) for n in range(32)]
    return tuple(op)


class _DeflateStream:
    """The ``<key>.npy`` member of a C-contiguous array as one raw deflate
    stream built as rows complete: the header, then the body in
    independently deflated pieces cut at ABSOLUTE multiples of _PIECE bytes
    (each ends on a sync flush, the last one finishes the stream -- pigz's
    layout), so the compressed bytes do not depend on the order or the
    grouping in which rows arrive (one process or the ranks of a sharded
    session write the same file).  A piece is deflated as soon as all its
    rows are in, wherever it lies; the CRC-32 is the pieces' CRCs combined in
    order at finish."""

    def __init__(self, arr: np.ndarray, level: int, pool):
        self.arr, self.level, self.pool = arr, level, pool
        head = _npy_header(arr)
        c = zlib.compressobj(level, zlib.DEFLATED, -15)
        self.head = c.compress(head) + c.flush(zlib.Z_SYNC_FLUSH)
        self.head_crc, self.head_size = zlib.crc32(head), len(head)
        self.rowbytes = arr[0].nbytes if arr.ndim and arr.shape[0] else 0
        self.nbytes = arr.nbytes if arr.ndim else 0
        self.npieces = self.nbytes // _PIECE  # whole pieces (the tail is deflated at finish)
        self.done: Dict[int, tuple] = {}      # piece -> (deflated bytes, crc)

    def _body(self) -> memoryview:
        return memoryview(self.arr.reshape(-1).view(np.uint8))

    def _rows_of(self, i: int):
        return (i * _PIECE) // self.rowbytes, ((i + 1) * _PIECE - 1) // self.rowbytes + 1

    def feed_rows(self, filled: np.ndarray, r0: int, r1: int) -> None:
        """Rows [r0, r1) were just written (`filled`: every final row): deflate
        the whole pieces they touch that are now complete."""
        if not self.rowbytes:
            return
        i0, i1 = (r0 * self.rowbytes) // _PIECE, min(self.npieces, (r1 * self.rowbytes - 1) // _PIECE + 1)
        todo = [i for i in range(i0, i1) if i not in self.done and filled[slice(*self._rows_of(i))].all()]
        if not todo:
            return
        body = self._body()
        res = self.pool.map(lambda i: (_deflate_one(body[i * _PIECE:(i + 1) * _PIECE], self.level, False),
                                       zlib.crc32(body[i * _PIECE:(i + 1) * _PIECE])), todo)
        for i, r in zip(todo, res):
            self.done[i] = r

    def feed(self, upto: int) -> None:
        """Rows [0, upto) are final."""
        if self.rowbytes and upto:
            self.feed_rows(np.arange(self.arr.shape[0]) < upto, 0, upto)

    def finish(self):
        body = self._body() if self.arr.ndim else memoryview(b"")
        missing = [i for i in range(self.npieces) if i not in self.done]
        if missing:
            res = self.pool.map(lambda i: (_deflate_one(body[i * _PIECE:(i + 1) * _PIECE], self.level, False),
                                           zlib.crc32(body[i * _PIECE:(i + 1) * _PIECE])), missing)
            for i, r in zip(missing, res):
                self.done[i] = r
        pieces, crc = [self.head], self.head_crc
        op = _crc_zeros_op(_PIECE) if self.npieces else None
        for i in range(self.npieces):
            z, c = self.done[i]
            pieces.append(z)
            crc = _gf2_times(op, crc) ^ c
        tail = body[self.npieces * _PIECE:]
        if len(tail):
            pieces.append(_deflate_one(tail, self.level, True))
            crc = _gf2_times(_crc_zeros_op(len(tail)), crc) ^ zlib.crc32(tail)
        else:
            pieces.append(zlib.compressobj(self.level, zlib.DEFLATED, -15).flush(zlib.Z_FINISH))
        return pieces, crc & 0xFFFFFFFF, self.head_size + self.nbytes


def save_npz(path: str, arrays: Dict[str, np.ndarray], level: int = 4, workers: int = 0,
             precompressed: Optional[dict] = None, pool=None) -> None:
    """np.savez_compressed's file (a zip of ``<key>.npy`` members, deflated;
    np.load reads it) written with the members' deflate streams compressed
    in parallel pieces.  Level 4 is h5py's gzip default, the reference's
    dataset compression (M/io/result.py:36-61).  Zip64 records are written
    when a size or offset needs them."""
    import concurrent.futures as cf
    if any(np.asarray(a).dtype.hasobject for a in arrays.values()):
        np.savez_compressed(path, **arrays)  # object arrays need np.save's pickling
        return
    precompressed = precompressed or {}
    workers = workers or max(1, min(16, len(os.sched_getaffinity(0))))
    M32 = 0xFFFFFFFF
    central = []
    own = pool is None
    pool = cf.ThreadPoolExecutor(workers) if own else pool
    def member(arr):
        a = np.asarray(arr)
        a = a if a.flags.c_contiguous else a.copy(order="C")  # (ascontiguousarray would make 0-d arrays 1-d)
        head = _npy_header(a)
        body = memoryview(a.reshape(-1).view(np.uint8)) if a.size else memoryview(b"")
        crc = zlib.crc32(body, zlib.crc32(head))
        size = len(head) + len(body)
        if size <= _PIECE:
            pieces = [_deflate_one(memoryview(head + bytes(body)), level, True)]
        else:  # header, then the body's pieces: one deflate stream
            c = zlib.compressobj(level, zlib.DEFLATED, -15)
            pieces = [c.compress(head) + c.flush(zlib.Z_SYNC_FLUSH)] + _deflate_pieces(body, level, pool)
        return pieces, crc, size

    # the small members (scalars, keypoints, metadata: one piece each) are
    # deflated concurrently, the large ones piecewise on the pool as they
    # come; the file is written in member order either way
    small = {k: pool.submit(member, v) for k, v in arrays.items()
             if k not in precompressed and len(_npy_header(np.asarray(v))) + np.asarray(v).nbytes <= _PIECE}
    with open(path, "wb") as fh:
        for key, arr in arrays.items():
            if key in precompressed:  # (pieces, crc, size) of a _DeflateStream
                pieces, crc, size = precompressed[key]
            elif key in small:
                pieces, crc, size = small[key].result()
            else:
                pieces, crc, size = member(arr)
            csize = sum(len(x) for x in pieces)
            name = (key + ".npy").encode()
            off = fh.tell()
            z64 = size >= _ZIP64_AT or csize >= _ZIP64_AT or off >= _ZIP64_AT
            extra = struct.pack("<HHQQ", 1, 16, size, csize) if z64 else b""
            fh.write(struct.pack("<IHHHHHIIIHH", 0x04034B50, 45 if z64 else 20, 0, 8, 0, 0x21, crc,
                                 M32 if z64 else csize, M32 if z64 else size, len(name), len(extra)))
            fh.write(name)
            fh.write(extra)
            for x in pieces:
                fh.write(x)
            central.append((name, crc, size, csize, off))
        cd_off = fh.tell()
        for name, crc, size, csize, off in central:
            z64 = size >= _ZIP64_AT or csize >= _ZIP64_AT or off >= _ZIP64_AT
            extra = struct.pack("<HHQQQ", 1, 24, size, csize, off) if z64 else b""
            fh.write(struct.pack("<IHHHHHHIIIHHHHHII", 0x02014B50, 45, 45 if z64 else 20, 0, 8, 0, 0x21, crc,
                                 M32 if z64 else csize, M32 if z64 else size, len(name), len(extra), 0, 0, 0,
                                 0o600 << 16, M32 if z64 else off))
            fh.write(name)
            fh.write(extra)
        cd_size = fh.tell() - cd_off
        n = len(central)
        if cd_off >= _ZIP64_AT or n >= 0xFFFF:
            z_off = fh.tell()
            fh.write(struct.pack("<IQHHIIQQQQ", 0x06064B50, 44, 45, 45, 0, 0, n, n, cd_size, cd_off))
            fh.write(struct.pack("<IIQI", 0x07064B50, 0, z_off, 1))
            fh.write(struct.pack("<IHHHHIIH", 0x06054B50, 0, 0, 0xFFFF, 0xFFFF, M32, M32, 0))
        else:
            fh.write(struct.pack("<IHHHHIIH", 0x06054B50, 0, 0, n, n, cd_size, cd_off, 0))
    if own:
        pool.shutdown()


def open_results(output_dir: str, bg_roi_index: int = 0):
    """results_XX.h5 via h5py when importable, else a MemoryH5 saved as
    results_XX.npz."""
    try:
        import h5py
    except ImportError:
        return MemoryH5(os.path.join(output_dir, f"results_{bg_roi_index:02d}.npz"))
    return h5py.File(os.path.join(output_dir, f"results_{bg_roi_index:02d}.h5"), mode="w")


def dict_to_h5(h5_file, data: dict, root: str = "/", annotations: Optional[dict] = None) -> None:
    """Nested dict -> datasets under `root`.  None becomes an empty
    variable-length string dataset (h5py.Empty; "" in a MemoryH5, which has
    no empty datasets).  As in the reference, a value that cannot be stored
    is logged and skipped, not raised: the parameters are metadata, and one
    odd entry must not fail the results file."""
    import logging
    if not root.endswith("/"):
        root = root + "/"
    annotations = annotations or {}
    for key, item in data.items():
        dest = root + key
        if isinstance(item, dict):
            dict_to_h5(h5_file, item, dest)
            continue
        try:
            if isinstance(item, (np.ndarray, np.int64, np.float64, str, bytes)):
                h5_file[dest] = item
            elif isinstance(item, (tuple, list)):
                h5_file[dest] = np.asarray(item)
            elif isinstance(item, (int, float)):
                h5_file[dest] = np.asarray([item])[0]
            elif item is None:
                if isinstance(h5_file, MemoryH5):
                    h5_file[dest] = ""
                else:
                    import h5py
                    h5_file.create_dataset(dest, data=h5py.Empty(dtype=h5py.special_dtype(vlen=str)))
            else:
                raise ValueError(f"Cannot save {type(item)} type to key {dest}")
        except Exception as exc:  # M/io/util.py:171-174
            logging.error(exc, exc_info=True)
            logging.error(f'h5py could not encode key: "{key}"')
            continue
        if key in annotations:
            h5_file[dest].attrs["description"] = "" if annotations[key] is None else annotations[key]


def create_extract_h5(h5_file, config_data: dict, status_dict: dict) -> None:
    """Datasets and metadata of an extraction result file (layout, dtypes and
    descriptions of M/io/result.py:14-103)."""
    nframes = config_data["nframes"]
    crop = config_data["crop_size"]
    h5_file.create_dataset("metadata/uuid", data=status_dict["uuid"])
    for name, desc in scalar_attributes().items():
        h5_file.create_dataset(f"scalars/{name}", (nframes,), "float32", compression="gzip")
        h5_file[f"scalars/{name}"].attrs["description"] = desc
    for name, desc in keypoint_attributes().items():
        h5_file.create_dataset(f"keypoints/{name}", (nframes,), "float32", compression="gzip")
        h5_file[f"keypoints/{name}"].attrs["description"] = desc
    h5_file.create_dataset("timestamps", compression="gzip", data=config_data["timestamps"])
    h5_file["timestamps"].attrs["description"] = "Depth video timestamps"
    h5_file.create_dataset("frames", (nframes, crop[0], crop[1]), config_data["frame_dtype"], compression="gzip")
    h5_file["frames"].attrs["description"] = "3D Numpy array of depth frames (nframes x w x h, in mm)"
    if config_data.get("use_tracking_model", False):
        h5_file.create_dataset("frames_mask", (nframes, crop[0], crop[1]), "float32", compression="gzip")
        h5_file["frames_mask"].attrs["description"] = "Log-likelihood values from the tracking model (nframes x w x h)"
    else:
        h5_file.create_dataset("frames_mask", (nframes, crop[0], crop[1]), "bool", compression="gzip")
        h5_file["frames_mask"].attrs["description"] = "Boolean mask, false=not mouse, true=mouse"
    if config_data.get("flip_classifier") is not None:
        h5_file.create_dataset("metadata/extraction/flips", (nframes,), "bool", compression="gzip")
        h5_file["metadata/extraction/flips"].attrs["description"] = \
            "Output from flip classifier, false=no flip, true=flip"
    h5_file.create_dataset("metadata/extraction/true_depth", data=config_data["true_depth"])
    h5_file["metadata/extraction/true_depth"].attrs["description"] = "Detected true depth of arena floor in mm"
    h5_file.create_dataset("metadata/extraction/roi", data=config_data["roi"], compression="gzip")
    h5_file["metadata/extraction/roi"].attrs["description"] = "ROI mask"
    h5_file.create_dataset("metadata/extraction/first_frame", data=config_data["first_frame"], compression="gzip")
    h5_file["metadata/extraction/first_frame"].attrs["description"] = "First frame of depth dataset"
    h5_file.create_dataset("metadata/extraction/background", data=config_data["bground_im"], compression="gzip")
    h5_file["metadata/extraction/background"].attrs["description"] = "Computed background image"
    h5_file.create_dataset("metadata/extraction/extract_version", data=PACKAGE_VERSION)
    h5_file["metadata/extraction/extract_version"].attrs["description"] = "Version of moseq2-extract"
    dict_to_h5(h5_file, status_dict.get("parameters", {}), "metadata/extraction/parameters")
    for key, value in status_dict.get("metadata", {}).items():
        if isinstance(value, list) and len(value) > 0 and isinstance(value[0], str):
            value = [v.encode("utf8") for v in value]
        if value is not None:
            h5_file.create_dataset(f"metadata/acquisition/{key}", data=value)
        else:
            h5_file.create_dataset(f"metadata/acquisition/{key}", dtype="f")


def write_extracted_chunk_to_h5(h5_file, results: dict) -> None:
    """Scalars, crops, masks, flips and keypoints of one chunk at rows
    results['frame_idxs'] (data sliced from results['offset'], as the
    reference does -- which requires offset 0 in practice)."""
    rows = results["frame_idxs"]
    off = results["offset"]
    for name, vals in results["scalars"].items():
        h5_file[f"scalars/{name}"][rows] = np.asarray(vals)[off:]
    h5_file["frames"][rows] = results["depth_frames"][off:]
    h5_file["frames_mask"][rows] = results["mask_frames"][off:]
    h5_file["metadata/extraction/flips"][rows] = np.asarray(results["features"]["flips"])[off:]
    for name, vals in results["keypoints"].items():
        h5_file[f"keypoints/{name}"][rows] = np.asarray(vals)[off:]
    hook = getattr(h5_file, "rows_written", None)
    if hook is not None:  # MemoryH5: deflate the completed rows now
        hook(rows)


class KeypointsTSVWriter:
    """keypoints_XX.tsv: Frame_Idx, Flip, Centroid_X, Centroid_Y, Angle, then
    every keypoint field, one row per frame, appended per chunk.  `path` /
    `header=False`: a headerless part file (one per rank of a sharded
    session, joined by join_tsv_parts)."""

    def __init__(self, output_dir: str, bg_roi_index: int = 0, path: Optional[str] = None, header: bool = True):
        self.path = path or os.path.join(output_dir, f"keypoints_{bg_roi_index:02d}.tsv")
        self._header = header
        self._fresh = True  # the first write truncates the file

    @staticmethod
    def columns(data: dict) -> dict:
        feats = data["features"]
        cen = np.asarray(feats["features"]["centroid"])
        cols = {"Frame_Idx": np.asarray(data["frame_idxs"]), "Flip": np.asarray(feats["flips"]),
                "Centroid_X": cen[:, 0], "Centroid_Y": cen[:, 1],
                "Angle": np.asarray(feats["features"]["orientation"])}
        for k, v in data["keypoints"].items():
            cols[k] = np.asarray(v)
        return cols

    def write(self, data: dict) -> None:
        cols = self.columns(data)
        # the bytes of pandas.DataFrame(cols).to_csv(sep="\t", index=False)
        # (shortest round-trip floats, NaN as an empty field): formatted in
        # libmdx's host code (no GIL held) when every column is float64 /
        # bool / integer, else here
        body = _tsv_rows_native(list(cols.values()))
        if body is None:
            cells = [_tsv_cells(v) for v in cols.values()]
            body = "".join("\t".join(r) + "\n" for r in zip(*cells)).encode()
        with open(self.path, "wb" if self._fresh else "ab") as fh:
            if self._header and self._fresh:
                fh.write(("\t".join(cols) + "\n").encode())
            fh.write(body)
        self._fresh = False


def join_tsv_parts(path: str, header_cols, parts) -> None:
    """keypoints_XX.tsv of a sharded session: the header, then the ranks'
    headerless part files in rank (= session) order; the parts are removed."""
    with open(path, "wb") as out:
        out.write(("\t".join(header_cols) + "\n").encode())
        for p in parts:
            if os.path.exists(p):
                with open(p, "rb") as fh:
                    while True:
                        b = fh.read(1 << 24)
                        if not b:
                            break
                        out.write(b)
                os.remove(p)


def _tsv_rows_native(columns) -> Optional[bytes]:
    """mdx_format_tsv_rows over the columns, or None when a column's dtype
    has no native form (float32 / float16: numpy's own shortest repr)."""
    import ctypes
    kinds, keep = [], []
    for a in columns:
        a = np.asarray(a)
        if a.dtype == np.float64:
            kinds.append(0)
            keep.append(np.ascontiguousarray(a))
        elif a.dtype == np.bool_:
            kinds.append(1)
            keep.append(np.ascontiguousarray(a).view(np.uint8))
        elif a.dtype.kind in "iu" and a.dtype.itemsize <= 8 and (a.dtype.kind == "i" or a.dtype.itemsize < 8):
            kinds.append(2)
            keep.append(np.ascontiguousarray(a, dtype=np.int64))
        else:
            return None
    n = len(keep[0]) if keep else 0
    if any(len(k) != n for k in keep):
        raise ValueError("keypoints TSV: columns of different lengths")
    from ._lib import call
    ptrs = (ctypes.c_void_p * len(keep))(*[k.ctypes.data for k in keep])
    kd = (ctypes.c_int * len(kinds))(*kinds)
    cap = n * (len(keep) * 40 + 1) + 1
    buf = ctypes.create_string_buffer(cap)
    nb = call("mdx_format_tsv_rows", ptrs, kd, len(keep), n, buf, cap)
    return buf.raw[:nb]


def _tsv_cells(a: np.ndarray) -> list:
    """One column's fields as pandas' to_csv writes them."""
    a = np.asarray(a)
    if a.dtype == np.bool_:
        return ["True" if v else "False" for v in a.tolist()]
    if a.dtype.kind in "iu":
        return [str(v) for v in a.tolist()]
    if a.dtype == np.float64:
        return ["" if v != v else repr(v) for v in a.tolist()]
    if a.dtype.kind == "f":  # float32 / float16: numpy's shortest repr of that width
        return ["" if v != v else str(v) for v in a]
    raise TypeError(f"keypoints TSV: unsupported column dtype {a.dtype}")


def _plain(v):
    """YAML-safe plain value (tuples -> lists, numpy scalars/arrays -> Python)."""
    if isinstance(v, dict):
        return {str(k): _plain(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_plain(x) for x in v]
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, np.generic):
        return v.item()
    return v


def status_filename(output_dir: str, bg_roi_index: int = 0) -> str:
    """results_XX.yaml next to the results (M/extract.py:48)."""
    return os.path.join(output_dir, f"results_{bg_roi_index:02d}.yaml")


def write_status(path: str, status: dict) -> None:
    """write_yaml (M/io/util.py:99-109): safe YAML, block style."""
    import yaml
    with open(path, "w", encoding="utf-8") as fh:
        yaml.safe_dump(_plain(status), fh, default_flow_style=False)


def check_completion_status(path: str) -> bool:
    """M/proc/util.py:63-77: True when the status file says complete."""
    if os.path.exists(path):
        import yaml
        with open(path, "r", encoding="utf-8") as fh:
            return bool(yaml.safe_load(fh)["complete"])
    return False
