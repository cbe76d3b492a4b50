"""kaarme_amd -- Python host mirror of the MI355X canonical k-mer counting engine.

Thin ctypes binding over ``lib/libkc.so`` (C ABI in ``include/kc_api.h``).  It mirrors
the reference's operator interface for the hot path: the ``parse_input_*`` functors
(``include/parallel_parser.hpp``) become :func:`count_file` / :class:`KmerCounter`,
``hash_kmers(chunk, format)`` becomes :meth:`KmerCounter.count_chunk`, the Bloom pass
``bloom_filter_kmers`` becomes :meth:`KmerCounter.bloom_chunk`, and the writers
(``write_kmers_on_disk_separately_even_faster`` / ``write_kmers``) become
:meth:`KmerCounter.write`.

There is no CPU fallback: if ``libkc.so`` is missing or no HIP device is usable, the
calls raise.  PyTorch is optional and only used by ``bench.py`` for device buffers,
streams and ``torch.distributed``.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# KC_LIB overrides the library (A/B runs of two builds); default: the in-tree build
LIB_PATH = os.environ.get("KC_LIB") or os.path.join(PKG_ROOT, "lib", "libkc.so")
CLI_PATH = os.path.join(PKG_ROOT, "bin", "kaarme")
GEN_PATH = os.path.join(PKG_ROOT, "bin", "kc_gen")

KC_OK = 0
ERRORS = {
    -1: "KC_ERR_ARG",
    -2: "KC_ERR_HIP",
    -3: "KC_ERR_TABLE_FULL",
    -4: "KC_ERR_STATE",
    -5: "KC_ERR_IO",
    -6: "KC_ERR_NOMEM",
    -7: "KC_ERR_UNSUPPORTED",
}
FMT_FASTA, FMT_FASTQ, FMT_PLAIN = 0, 1, 2

# Public C-ABI symbols (include/kc_api.h); tests check every one is exported.
EXPORTS = (
    "kc_create", "kc_destroy", "kc_last_error", "kc_bloom_chunk", "kc_bloom_finalize",
    "kc_count_chunk", "kc_bloom_device", "kc_count_device", "kc_sync", "kc_finish", "kc_dump",
    "kc_write", "kc_key_words", "kc_free", "kc_plan_chunks", "kc_synth_bytes", "kc_synth_device",
    "kc_reset", "kc_profile", "kc_get_timing", "kc_route_device", "kc_insert_keys_device",
    "kc_route_table_device", "kc_route_hint", "kc_insert_counts_device", "kc_clear_table", "kc_insert_counts_runs_device",
    "kc_xxh64", "kc_bloom_info", "kc_bloom_read", "kc_bloom_write", "kc_synth_skew_device",
    "kc_table_size_reference", "kc_bloom_get_device", "kc_bloom_merge_device", "kc_bloom_set_device",
    "kc_bloom_estimate", "kc_compact", "kc_compact_dump", "kc_compact_lookup", "kc_compact_read", "kc_size_table",
    "kc_estimate_distinct_device", "kc_bloom_records_device", "kc_count_records_device", "kc_plan_chunks_device",
    "kc_output_digest", "kc_route_superkmers_device", "kc_count_packed_device", "kc_bloom_packed_device",
)


class KcError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class kc_config(ctypes.Structure):
    _fields_ = [
        ("k", ctypes.c_int32), ("mode", ctypes.c_int32), ("bf_enable", ctypes.c_int32),
        ("device", ctypes.c_int32), ("table_slots", ctypes.c_uint64), ("est_unique", ctypes.c_uint64),
        ("fpr", ctypes.c_double), ("min_abundance", ctypes.c_uint64), ("batch_bytes", ctypes.c_uint64),
    ]


class kc_chunk(ctypes.Structure):
    _fields_ = [("off", ctypes.c_uint64), ("len", ctypes.c_uint64),
                ("broken_header", ctypes.c_int32), ("pad", ctypes.c_int32)]


class kc_timing(ctypes.Structure):
    _fields_ = [("gather_ms", ctypes.c_double), ("tokenize_ms", ctypes.c_double), ("count_ms", ctypes.c_double),
                ("launches", ctypes.c_uint64), ("symbols", ctypes.c_uint64)]


class kc_synth_skew(ctypes.Structure):
    _fields_ = [("homo_frac", ctypes.c_double), ("dinuc_frac", ctypes.c_double),
                ("repeat_len", ctypes.c_uint32), ("repeat_copies", ctypes.c_uint32)]


class kc_compact_info(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("slots", "kmers", "chain_starts", "bytes", "table_bytes")]


class kc_digest(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("lines", "count_sum", "hash_sum", "hash_xor")]


class kc_stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "windows", "inserted", "distinct", "table_slots", "bf_windows", "bf_bits", "new_in_first",
        "new_in_second", "failed_in_first", "chunks", "bytes", "part_fallbacks", "spilled", "heavy_records",
        "reused_passes", "reuse_level", "route_counts_kept", "deferred_level3")]

    def as_dict(self) -> dict:
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


_lib: Optional[ctypes.CDLL] = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libkc.so (raises if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise FileNotFoundError(
            f"{path} not built; run `make -C {PKG_ROOT}` or __graft_entry__.build()")
    # PyTorch-ROCm wheels ship their own libamdhip64.so.7.  If torch is around, load
    # it first so that libkc.so binds to that same runtime (one HIP runtime per
    # process; device pointers and streams are then shared with torch).  Without
    # torch, libkc.so uses /opt/rocm's runtime through its RUNPATH.
    try:
        import torch  # noqa: F401
        if torch.cuda.is_available():
            torch.cuda.init()
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    P, U64, I32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
    sig = {
        "kc_create": (I32, [ctypes.POINTER(kc_config), ctypes.POINTER(P)]),
        "kc_destroy": (None, [P]),
        "kc_last_error": (ctypes.c_char_p, [P]),
        "kc_bloom_chunk": (I32, [P, P, ctypes.c_size_t, I32, I32]),
        "kc_bloom_finalize": (I32, [P, ctypes.POINTER(U64)]),
        "kc_count_chunk": (I32, [P, P, ctypes.c_size_t, I32, I32]),
        "kc_bloom_device": (I32, [P, P, ctypes.POINTER(kc_chunk), ctypes.c_size_t, I32, P]),
        "kc_count_device": (I32, [P, P, ctypes.POINTER(kc_chunk), ctypes.c_size_t, I32, P]),
        "kc_estimate_distinct_device": (I32, [P, P, ctypes.POINTER(kc_chunk), ctypes.c_size_t, I32, P,
                                              ctypes.POINTER(ctypes.c_double)]),
        "kc_size_table": (I32, [P, U64]),
        "kc_route_superkmers_device": (I32, [P, P, ctypes.POINTER(kc_chunk), ctypes.c_size_t, I32, ctypes.c_uint32,
                                             I32, P, P, U64, ctypes.POINTER(U64), ctypes.POINTER(U64), P]),
        "kc_count_packed_device": (I32, [P, P, P, U64, U64, P]),
        "kc_bloom_packed_device": (I32, [P, P, P, U64, U64, P]),
        "kc_sync": (I32, [P]),
        "kc_finish": (I32, [P, ctypes.POINTER(kc_stats)]),
        "kc_dump": (I32, [P, ctypes.POINTER(ctypes.POINTER(U64)), ctypes.POINTER(U64)]),
        "kc_write": (I32, [P, ctypes.c_char_p]),
        "kc_output_digest": (I32, [P, ctypes.POINTER(kc_digest)]),
        "kc_key_words": (I32, [P]),
        "kc_free": (None, [P]),
        "kc_plan_chunks": (I32, [P, U64, I32, U64, I32, ctypes.POINTER(ctypes.POINTER(kc_chunk)),
                                 ctypes.POINTER(U64)]),
        "kc_plan_chunks_device": (I32, [P, U64, I32, U64, I32, ctypes.POINTER(ctypes.POINTER(kc_chunk)),
                                 ctypes.POINTER(U64)]),
        "kc_synth_bytes": (U64, [U64, U64, ctypes.c_uint32, ctypes.c_uint32]),
        "kc_reset": (I32, [P]),
        "kc_clear_table": (I32, [P]),
        "kc_insert_counts_runs_device": (I32, [P, P, ctypes.POINTER(U64), ctypes.c_uint32, P]),
        "kc_route_device": (I32, [P, P, ctypes.POINTER(kc_chunk), ctypes.c_size_t, I32, ctypes.c_uint32, P, U64,
                                  ctypes.POINTER(U64), P]),
        "kc_insert_keys_device": (I32, [P, P, U64, P]),
        "kc_route_table_device": (I32, [P, ctypes.c_uint32, P, U64, P, P]),
        "kc_route_hint": (I32, [P, ctypes.c_uint32]),
        "kc_insert_counts_device": (I32, [P, P, U64, P]),
        "kc_bloom_records_device": (I32, [P, P, U64, P]),
        "kc_count_records_device": (I32, [P, P, U64, P]),
        "kc_profile": (I32, [P, I32]),
        "kc_get_timing": (I32, [P, ctypes.POINTER(kc_timing)]),
        "kc_synth_device": (I32, [P, U64, U64, U64, U64, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.c_double, ctypes.c_double, P]),
        "kc_xxh64": (I32, [P, P, U64, P]),
        "kc_table_size_reference": (U64, [U64]),
        "kc_synth_skew_device": (I32, [P, U64, U64, U64, U64, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_double, ctypes.c_double, ctypes.POINTER(kc_synth_skew), P]),
        "kc_bloom_info": (I32, [P, ctypes.POINTER(U64), ctypes.POINTER(U64), ctypes.POINTER(I32),
                                ctypes.POINTER(I32), ctypes.POINTER(I32)]),
        "kc_bloom_read": (I32, [P, P, U64]),
        "kc_bloom_write": (I32, [P, P, U64]),
        "kc_bloom_get_device": (I32, [P, P, U64, U64, P]),
        "kc_bloom_merge_device": (I32, [P, P, ctypes.c_uint32, U64, P, P]),
        "kc_bloom_set_device": (I32, [P, P, U64, ctypes.POINTER(U64), P]),
        "kc_bloom_estimate": (I32, [P, ctypes.POINTER(U64), P]),
        "kc_compact": (I32, [P, ctypes.c_double, ctypes.POINTER(kc_compact_info)]),
        "kc_compact_dump": (I32, [P, ctypes.POINTER(ctypes.POINTER(U64)), ctypes.POINTER(U64), ctypes.POINTER(U64),
                                  ctypes.POINTER(ctypes.c_double)]),
        "kc_compact_lookup": (I32, [P, P, U64, P]),
        "kc_compact_read": (I32, [P, P, U64, P, U64]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


MAX_K = 479  # include/kc_api.h KC_MAX_K


def words_for_k(k: int) -> int:
    return k // 32 + 1


def xxh64_device(values: Sequence[int], seeds: Sequence[int]) -> List[int]:
    """XXH64(&v, 8, seed) of each pair by the device function of the reference-layout
    Bloom passes (kc_xxh64 test hook)."""
    lib = load_library()
    v = np.ascontiguousarray(values, dtype=np.uint64)
    sd = np.ascontiguousarray(seeds, dtype=np.uint64)
    out = np.zeros(v.size, dtype=np.uint64)
    rc = lib.kc_xxh64(v.ctypes.data, sd.ctypes.data, v.size, out.ctypes.data)
    if rc:
        raise KcError(rc, "kc_xxh64")
    return [int(x) for x in out]


def detect_format(path: str, first_byte: int) -> int:
    """file_format (main.cpp:27-68) on an uncompressed image: returns FMT_* or raises."""
    ext = os.path.splitext(path)[1]
    if ext in (".fasta", ".fa"):
        ok, fmt = first_byte == ord(">"), FMT_FASTA
    elif ext in (".fastq", ".fq"):
        ok, fmt = first_byte == ord("@"), FMT_FASTQ
    else:
        ok, fmt = first_byte in b"actgACGT", FMT_PLAIN
    if not ok:
        raise ValueError(f"Input file {path} is ill-formed")
    return fmt


def plan_chunks(image: bytes, k: int, fmt: int, chunk_size: int = 0) -> List[Tuple[int, int, int]]:
    """Reference chunk table (off, len, broken_header) of a file image."""
    lib = load_library()
    buf = ctypes.create_string_buffer(bytes(image), len(image)) if len(image) else None
    out = ctypes.POINTER(kc_chunk)()
    n = ctypes.c_uint64()
    rc = lib.kc_plan_chunks(buf, len(image), k, chunk_size, fmt, ctypes.byref(out), ctypes.byref(n))
    if rc:
        raise KcError(rc, "kc_plan_chunks")
    res = [(out[i].off, out[i].len, out[i].broken_header) for i in range(n.value)]
    lib.kc_free(out)
    return res


def plan_chunks_device(dev_ptr: int, size: int, k: int, fmt: int, chunk_size: int = 0) -> List[Tuple[int, int, int]]:
    """plan_chunks for an image in device memory (kc_plan_chunks_device: only the bytes around
    chunk ends are copied to the host)."""
    lib = load_library()
    out = ctypes.POINTER(kc_chunk)()
    n = ctypes.c_uint64()
    rc = lib.kc_plan_chunks_device(ctypes.c_void_p(dev_ptr or None), size, k, chunk_size, fmt, ctypes.byref(out),
                                   ctypes.byref(n))
    if rc:
        raise KcError(rc, "kc_plan_chunks_device")
    res = [(out[i].off, out[i].len, out[i].broken_header) for i in range(n.value)]
    lib.kc_free(out)
    return res


def decode_records(records: np.ndarray, k: int) -> List[Tuple[str, int]]:
    """(W+1)-word records -> [(kmer string, T(c))] (test helper, vectorised)."""
    W = words_for_k(k)
    recs = records.reshape(-1, W + 1)
    n = recs.shape[0]
    chars = np.empty((n, k), dtype=np.uint8)
    lut = np.frombuffer(b"ACGT", dtype=np.uint8)
    for j in range(k):
        bit = 2 * (k - 1 - j)
        word = W - 1 - bit // 64
        chars[:, j] = lut[(recs[:, word] >> np.uint64(bit % 64)) & np.uint64(3)]
    strs = [bytes(r).decode() for r in chars]
    return list(zip(strs, (int(c) for c in recs[:, W])))


@dataclass
class Config:
    k: int
    mode: int = 2
    table_slots: int = 1 << 20
    bf_enable: bool = False
    est_unique: int = 0
    fpr: float = 0.01
    min_abundance: int = 2
    device: int = 0
    batch_bytes: int = 0

    def to_c(self) -> kc_config:
        return kc_config(self.k, self.mode, int(self.bf_enable), self.device, self.table_slots,
                         self.est_unique, self.fpr, self.min_abundance, self.batch_bytes)


class KmerCounter:
    """One device table (+ optional double Bloom filter) behind the C ABI."""

    def __init__(self, cfg: Config):
        self.lib = load_library()
        self.cfg = cfg
        self._ctx = ctypes.c_void_p()
        c = cfg.to_c()
        rc = self.lib.kc_create(ctypes.byref(c), ctypes.byref(self._ctx))
        if rc:
            raise KcError(rc, self.lib.kc_last_error(None).decode())

    # -- lifecycle
    def close(self):
        if self._ctx:
            self.lib.kc_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc: int, what: str):
        if rc:
            raise KcError(rc, f"{what}: {self.lib.kc_last_error(self._ctx).decode()}")

    # -- passes over host chunks
    def bloom_chunk(self, buf: bytes, fmt: int, broken_header: bool = False):
        self._chk(self.lib.kc_bloom_chunk(self._ctx, buf, len(buf), fmt, int(broken_header)), "kc_bloom_chunk")

    def bloom_finalize(self) -> int:
        n = ctypes.c_uint64()
        self._chk(self.lib.kc_bloom_finalize(self._ctx, ctypes.byref(n)), "kc_bloom_finalize")
        return n.value

    def count_chunk(self, buf: bytes, fmt: int, broken_header: bool = False):
        self._chk(self.lib.kc_count_chunk(self._ctx, buf, len(buf), fmt, int(broken_header)), "kc_count_chunk")

    # -- passes over a device-resident image (e.g. a torch uint8 CUDA tensor's data_ptr)
    @staticmethod
    def _chunk_array(chunks: Sequence[Tuple[int, int, int]]):
        arr = (kc_chunk * max(1, len(chunks)))()
        for i, (o, l, b) in enumerate(chunks):
            arr[i].off, arr[i].len, arr[i].broken_header = o, l, b
        return arr

    def bloom_device(self, dev_ptr: int, chunks, fmt: int, stream: int = 0):
        arr = self._chunk_array(chunks)
        self._chk(self.lib.kc_bloom_device(self._ctx, ctypes.c_void_p(dev_ptr), arr, len(chunks), fmt,
                                           ctypes.c_void_p(stream or None)), "kc_bloom_device")

    def count_device(self, dev_ptr: int, chunks, fmt: int, stream: int = 0):
        arr = self._chunk_array(chunks)
        self._chk(self.lib.kc_count_device(self._ctx, ctypes.c_void_p(dev_ptr), arr, len(chunks), fmt,
                                           ctypes.c_void_p(stream or None)), "kc_count_device")

    def estimate_distinct_device(self, dev_ptr: int, chunks, fmt: int, stream: int = 0) -> float:
        """HyperLogLog estimate of the image's distinct canonical k-mers (2^14 registers, ~0.8 %
        standard error); counts nothing.  For sizing a table before counting."""
        arr = self._chunk_array(chunks)
        est = ctypes.c_double(0.0)
        self._chk(self.lib.kc_estimate_distinct_device(self._ctx, ctypes.c_void_p(dev_ptr), arr, len(chunks), fmt,
                                                       ctypes.c_void_p(stream or None), ctypes.byref(est)),
                  "kc_estimate_distinct_device")
        return est.value

    def size_table(self, slots: int):
        """Size the table of the job about to be counted for `slots` k-mers (e.g. 1.1 x the distinct
        estimate) instead of -s, which stays the job's reference capacity; 0 = back to -s
        (kc_size_table: after create / reset, before the first counting pass)."""
        self._chk(self.lib.kc_size_table(self._ctx, int(slots)), "kc_size_table")

    def route_superkmers_device(self, dev_ptr: int, chunks, fmt: int, nshards: int, pk_ptr: int = 0, bk_ptr: int = 0,
                                cap_words: int = 0, m: int = 0, stream: int = 0):
        """Super-k-mers of a device image, per owner (canonical-minimizer owner, kc_api.h): region o of
        pk / bk (cap_words words each, at o * cap_words) receives owner o's packed stream.  Returns
        (words per owner, windows per owner); cap_words = 0 only sizes them.  Raises KcError
        (KC_ERR_NOMEM) when a region is too small -- its .words holds the sizes needed."""
        arr = self._chunk_array(chunks)
        words = (ctypes.c_uint64 * nshards)()
        wins = (ctypes.c_uint64 * nshards)()
        rc = self.lib.kc_route_superkmers_device(self._ctx, ctypes.c_void_p(dev_ptr), arr, len(chunks), fmt, nshards, m,
                                                 ctypes.c_void_p(pk_ptr or None), ctypes.c_void_p(bk_ptr or None),
                                                 cap_words, words, wins, ctypes.c_void_p(stream or None))
        if rc:
            err = KcError(rc, f"kc_route_superkmers_device: {self.lib.kc_last_error(self._ctx).decode()}")
            err.words = list(words)
            raise err
        return list(words), list(wins)

    def count_packed_device(self, pk_ptr: int, bk_ptr: int, n_words: int, windows: int = 0, stream: int = 0):
        """Counts the windows of a packed symbol stream in HBM (e.g. received super-k-mers)."""
        self._chk(self.lib.kc_count_packed_device(self._ctx, ctypes.c_void_p(pk_ptr or None),
                                                  ctypes.c_void_p(bk_ptr or None), n_words, windows,
                                                  ctypes.c_void_p(stream or None)), "kc_count_packed_device")

    def bloom_packed_device(self, pk_ptr: int, bk_ptr: int, n_words: int, windows: int = 0, stream: int = 0):
        """Bloom pass 1 over a packed symbol stream in HBM."""
        self._chk(self.lib.kc_bloom_packed_device(self._ctx, ctypes.c_void_p(pk_ptr or None),
                                                  ctypes.c_void_p(bk_ptr or None), n_words, windows,
                                                  ctypes.c_void_p(stream or None)), "kc_bloom_packed_device")

    def route_device(self, dev_ptr: int, chunks, fmt: int, nshards: int, out_ptr: int, out_capacity: int,
                     stream: int = 0) -> List[int]:
        """Table keys of the image's windows grouped by owner shard into out_ptr; returns counts."""
        arr = self._chunk_array(chunks)
        counts = (ctypes.c_uint64 * nshards)()
        self._chk(self.lib.kc_route_device(self._ctx, ctypes.c_void_p(dev_ptr), arr, len(chunks), fmt, nshards,
                                           ctypes.c_void_p(out_ptr), out_capacity, counts,
                                           ctypes.c_void_p(stream or None)), "kc_route_device")
        return [int(x) for x in counts]

    def insert_keys_device(self, keys_ptr: int, n_keys: int, stream: int = 0):
        self._chk(self.lib.kc_insert_keys_device(self._ctx, ctypes.c_void_p(keys_ptr), n_keys,
                                                 ctypes.c_void_p(stream or None)), "kc_insert_keys_device")

    def route_table_device(self, nshards: int, out_ptr: int, out_capacity: int, stream: int = 0) -> List[int]:
        """The table's occupied slots as {W table-key words, raw count} records grouped by
        owner shard into out_ptr (0 = count only); returns the per-owner record counts."""
        counts = (ctypes.c_uint64 * nshards)()
        self._chk(self.lib.kc_route_table_device(self._ctx, nshards, ctypes.c_void_p(out_ptr or None), out_capacity,
                                                 counts, ctypes.c_void_p(stream or None)), "kc_route_table_device")
        return [int(x) for x in counts]

    def route_hint(self, nshards: int):
        """The table will be routed to nshards owners: the counting passes keep the per-block
        owner counts so route_table_device runs no count pass (include/kc_api.h kc_route_hint)."""
        self._chk(self.lib.kc_route_hint(self._ctx, nshards), "kc_route_hint")

    def bloom_records_device(self, rec_ptr: int, n_records: int, stream: int = 0):
        """Bloom pass 1 over {key, count} records (include/kc_api.h kc_bloom_records_device)."""
        self._chk(self.lib.kc_bloom_records_device(self._ctx, ctypes.c_void_p(rec_ptr), n_records,
                                                   ctypes.c_void_p(stream or None)), "kc_bloom_records_device")

    def count_records_device(self, rec_ptr: int, n_records: int, stream: int = 0):
        """The counting pass over {key, count} records behind the gate (kc_count_records_device)."""
        self._chk(self.lib.kc_count_records_device(self._ctx, ctypes.c_void_p(rec_ptr), n_records,
                                                   ctypes.c_void_p(stream or None)), "kc_count_records_device")

    def insert_counts_device(self, rec_ptr: int, n_records: int, stream: int = 0):
        self._chk(self.lib.kc_insert_counts_device(self._ctx, ctypes.c_void_p(rec_ptr), n_records,
                                                   ctypes.c_void_p(stream or None)), "kc_insert_counts_device")

    def insert_counts_runs_device(self, rec_ptr: int, group_counts: Sequence[int], stream: int = 0):
        """Records in per-sender groups, each in kc_route_table_device order."""
        arr = (ctypes.c_uint64 * len(group_counts))(*group_counts)
        self._chk(self.lib.kc_insert_counts_runs_device(self._ctx, ctypes.c_void_p(rec_ptr), arr, len(group_counts),
                                                        ctypes.c_void_p(stream or None)),
                  "kc_insert_counts_runs_device")

    def key_words(self) -> int:
        return self.lib.kc_key_words(self._ctx)

    # -- Bloom filter test hooks (kc_bloom_info / kc_bloom_read / kc_bloom_write)
    def bloom_info(self) -> dict:
        nw, bits = ctypes.c_uint64(), ctypes.c_uint64()
        nh, ng, lay = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self._chk(self.lib.kc_bloom_info(self._ctx, ctypes.byref(nw), ctypes.byref(bits), ctypes.byref(nh),
                                         ctypes.byref(ng), ctypes.byref(lay)), "kc_bloom_info")
        return {"words": nw.value, "bits": bits.value, "nh": nh.value, "nh_gate": ng.value,
                "layout": "blocked" if lay.value else "reference"}

    def bloom_read(self) -> np.ndarray:
        n = self.bloom_info()["words"]
        a = np.zeros(n, dtype=np.uint32)
        self._chk(self.lib.kc_bloom_read(self._ctx, a.ctypes.data, n), "kc_bloom_read")
        return a

    def bloom_write(self, words: np.ndarray):
        a = np.ascontiguousarray(words, dtype=np.uint32)
        self._chk(self.lib.kc_bloom_write(self._ctx, a.ctypes.data, a.size), "kc_bloom_write")

    # -- sharded Bloom filter (kc_bloom_get/merge/set_device, kc_bloom_estimate)
    def bloom_get_device(self, dst_ptr: int, first_word: int, n_words: int, stream: int = 0):
        self._chk(self.lib.kc_bloom_get_device(self._ctx, ctypes.c_void_p(dst_ptr), first_word, n_words,
                                               ctypes.c_void_p(stream or None)), "kc_bloom_get_device")

    def bloom_merge_device(self, parts_ptr: int, nparts: int, n_words: int, out_ptr: int, stream: int = 0):
        self._chk(self.lib.kc_bloom_merge_device(self._ctx, ctypes.c_void_p(parts_ptr), nparts, n_words,
                                                 ctypes.c_void_p(out_ptr), ctypes.c_void_p(stream or None)),
                  "kc_bloom_merge_device")

    def bloom_set_device(self, src_ptr: int, n_words: int, stream: int = 0) -> int:
        """Install a whole filter; returns the new_in_second estimate the table is sized from."""
        n = ctypes.c_uint64()
        self._chk(self.lib.kc_bloom_set_device(self._ctx, ctypes.c_void_p(src_ptr), n_words, ctypes.byref(n),
                                               ctypes.c_void_p(stream or None)), "kc_bloom_set_device")
        return n.value

    def bloom_estimate(self, stream: int = 0) -> int:
        n = ctypes.c_uint64()
        self._chk(self.lib.kc_bloom_estimate(self._ctx, ctypes.byref(n), ctypes.c_void_p(stream or None)),
                  "kc_bloom_estimate")
        return n.value

    def sync(self):
        self._chk(self.lib.kc_sync(self._ctx), "kc_sync")

    def reset(self):
        self._chk(self.lib.kc_reset(self._ctx), "kc_reset")

    def clear_table(self):
        """Empty the table, keep the job's counters (kc_clear_table)."""
        self._chk(self.lib.kc_clear_table(self._ctx), "kc_clear_table")

    def profile(self, enable: bool = True):
        self._chk(self.lib.kc_profile(self._ctx, int(enable)), "kc_profile")

    def timing(self) -> dict:
        t = kc_timing()
        self._chk(self.lib.kc_get_timing(self._ctx, ctypes.byref(t)), "kc_get_timing")
        return {n: getattr(t, n) for n, _ in t._fields_}

    def finish(self) -> dict:
        st = kc_stats()
        self._chk(self.lib.kc_finish(self._ctx, ctypes.byref(st)), "kc_finish")
        return st.as_dict()

    # -- results
    def dump(self) -> np.ndarray:
        """Records as a uint64 array of shape (n, W+1): key words then T(c)."""
        p = ctypes.POINTER(ctypes.c_uint64)()
        n = ctypes.c_uint64()
        self._chk(self.lib.kc_dump(self._ctx, ctypes.byref(p), ctypes.byref(n)), "kc_dump")
        W = self.lib.kc_key_words(self._ctx)
        try:
            if n.value == 0:
                return np.zeros((0, W + 1), dtype=np.uint64)
            arr = np.ctypeslib.as_array(p, shape=(n.value * (W + 1),)).copy()
        finally:
            self.lib.kc_free(p)
        return arr.reshape(-1, W + 1)

    # -- Kaarme's compact representation (kc_compact*)
    def compact(self, load: float = 0.0) -> dict:
        """Build the compact slot words from the counted table; returns kc_compact_info."""
        info = kc_compact_info()
        self._chk(self.lib.kc_compact(self._ctx, load, ctypes.byref(info)), "kc_compact")
        return {n: getattr(info, n) for n, _ in kc_compact_info._fields_}

    def compact_dump(self):
        """(records (n, W+1) as dump(), longest walk, mean walk) reconstructed from the compact words."""
        p = ctypes.POINTER(ctypes.c_uint64)()
        n, mx, mean = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_double()
        self._chk(self.lib.kc_compact_dump(self._ctx, ctypes.byref(p), ctypes.byref(n), ctypes.byref(mx),
                                           ctypes.byref(mean)), "kc_compact_dump")
        W = self.lib.kc_key_words(self._ctx)
        try:
            arr = (np.ctypeslib.as_array(p, shape=(n.value * (W + 1),)).copy() if n.value
                   else np.zeros(0, dtype=np.uint64))
        finally:
            self.lib.kc_free(p)
        return arr.reshape(-1, W + 1), mx.value, mean.value

    def compact_lookup(self, keys: np.ndarray) -> np.ndarray:
        """T(c) of canonical keys (n, W) uint64 (dump's key layout) from the compact words; 0 = absent."""
        k = np.ascontiguousarray(keys, dtype=np.uint64)
        out = np.zeros(k.shape[0], dtype=np.uint32)
        self._chk(self.lib.kc_compact_lookup(self._ctx, k.ctypes.data, k.shape[0], out.ctypes.data),
                  "kc_compact_lookup")
        return out

    def compact_read(self, info: dict):
        """(slot words, secondary-array words) as uint64 arrays."""
        W = self.lib.kc_key_words(self._ctx)
        words = np.zeros(info["slots"], dtype=np.uint64)
        second = np.zeros(info["chain_starts"] * W, dtype=np.uint64)
        self._chk(self.lib.kc_compact_read(self._ctx, words.ctypes.data, words.size, second.ctypes.data,
                                           second.size), "kc_compact_read")
        return words, second.reshape(-1, W)

    def lines(self) -> List[str]:
        """Sorted "<KMER> <count>" lines (what sort(kaarme output) yields)."""
        return sorted(f"{s} {c}" for s, c in decode_records(self.dump(), self.cfg.k))

    def write(self, path: str):
        self._chk(self.lib.kc_write(self._ctx, path.encode()), "kc_write")

    def output_digest(self) -> dict:
        """Order-independent digest of the output text (kc_output_digest): lines, sum of T(c), and
        the sum mod 2^64 / XOR of XXH64 over every line (hash_sum / hash_xor as 16 hex digits, the
        format of oracle/kc_digest.c and tests/golden/fullsize.json)."""
        d = kc_digest()
        self._chk(self.lib.kc_output_digest(self._ctx, ctypes.byref(d)), "kc_output_digest")
        return digest_dict(d.lines, d.count_sum, d.hash_sum, d.hash_xor)


def digest_dict(lines: int, count_sum: int, hash_sum: int, hash_xor: int) -> dict:
    return {"lines": int(lines), "count_sum": int(count_sum), "hash_sum": f"{int(hash_sum) & (2**64 - 1):016x}",
            "hash_xor": f"{int(hash_xor) & (2**64 - 1):016x}"}


def combine_digests(parts: Iterable[dict]) -> dict:
    """The digest of the union of disjoint line sets (e.g. the owners of a sharded job)."""
    n = c = s = x = 0
    for d in parts:
        n += d["lines"]
        c += d["count_sum"]
        s += int(d["hash_sum"], 16)
        x ^= int(d["hash_xor"], 16)
    return digest_dict(n, c, s, x)


def same_digest(a: dict, b: dict) -> bool:
    return all(a[key] == b[key] for key in ("lines", "count_sum", "hash_sum", "hash_xor"))


def count_file(path: str, k: int, mode: int = 2, min_abundance: int = 2, table_slots: int = 1 << 20,
               bf_enable: bool = False, est_unique: int = 0, fpr: float = 0.01, chunk_size: int = 0,
               batch_bytes: int = 0, device: int = 0) -> Tuple[KmerCounter, dict]:
    """The parse_input_* functor chain (main.cpp:427-543) on one device, host chunks."""
    with open(path, "rb") as f:
        image = f.read()
    fmt = detect_format(path, image[0] if image else 0)
    chunks = plan_chunks(image, k, fmt, chunk_size)
    if not batch_bytes:  # a small input gets a stage of its own size (one batch, little pinned memory)
        staged = 4096 + sum((ln + 4095) // 4096 * 4096 for _, ln, _ in chunks)
        batch_bytes = staged if staged <= (256 << 20) else 0
    kc = KmerCounter(Config(k=k, mode=mode, table_slots=table_slots, bf_enable=bf_enable,
                            est_unique=est_unique, fpr=fpr, min_abundance=min_abundance,
                            batch_bytes=batch_bytes, device=device))
    mv = memoryview(image)
    if bf_enable:
        for off, ln, bh in chunks:
            kc.bloom_chunk(bytes(mv[off:off + ln]), fmt, bool(bh))
        kc.bloom_finalize()
    for off, ln, bh in chunks:
        kc.count_chunk(bytes(mv[off:off + ln]), fmt, bool(bh))
    stats = kc.finish()
    return kc, stats
