"""Device-resident batches for the MI355X engine.

PyTorch is used only as plumbing: it allocates HBM (``torch.empty(..., device="cuda")``) and
provides the HIP stream handle; every byte of CDC/fingerprint work runs in the engine's own HIP
kernels through the C-ABI (``sdfs_cdc_run_device``).

Synthetic workload (BASELINE.json configs[1]): ``n_streams`` independent write
streams of ``stream_bytes`` each, cut into CHUNK_LENGTH write buffers exactly as
DedupFileChannel.writeFile does (DedupFileChannel.java:310-338); every buffer is chunked from a
fresh CDC state.  Byte ``o`` of stream ``s`` is the counter-based SplitMix64 byte of
``oracle/cdc_ref.c:cdc_ref_synth`` (generated on the GPU by ``sdfs_cdc_synth_device``).
"""
from __future__ import annotations

from dataclasses import dataclass

from . import _lib
from .engine import HipVariableSha256HashEngine

SYNTH_SEED = 0x5DF50001


@dataclass
class DeviceBatch:
    engine: HipVariableSha256HashEngine
    nbuf: int
    buf_len: int
    device: str = "cuda:0"
    records: bool = True

    def __post_init__(self):
        import torch

        self.torch = torch
        dev = torch.device(self.device)
        if self.buf_len % 64:
            raise ValueError("buffer length must be a multiple of 64")
        self.cap = self.engine.slot_cap(self.buf_len)
        nslots = self.nbuf * self.cap
        self.data = torch.empty(self.nbuf * self.buf_len, dtype=torch.uint8, device=dev)
        self.counts = torch.zeros(self.nbuf, dtype=torch.int32, device=dev)
        self.starts = torch.zeros(nslots, dtype=torch.int32, device=dev)
        self.lens = torch.zeros(nslots, dtype=torch.int32, device=dev)
        self.digests = torch.zeros(nslots * 32, dtype=torch.uint8, device=dev)
        self.total = torch.zeros(1, dtype=torch.int32, device=dev)
        self.recs = (torch.zeros(nslots * _lib.RECORD_BYTES, dtype=torch.uint8, device=dev)
                     if self.records else None)
        self.out = _lib.DevOut(
            counts=self.counts.data_ptr(), starts=self.starts.data_ptr(), lens=self.lens.data_ptr(),
            digests=self.digests.data_ptr(), cap=self.cap, reserved=0,
            records=self.recs.data_ptr() if self.recs is not None else None,
            records_cap=nslots if self.recs is not None else 0, total=self.total.data_ptr())

    def set_records(self, table) -> None:
        """Have the engine write the fingerprint records straight into ``table`` (a [>= nbuf*cap,
        48] uint8 device tensor, e.g. a :class:`sdfs_amd.dist.RecordExchange` slot) instead of this
        batch's own record buffer: the exchange then all-gathers them with no snapshot copy."""
        rows = table.shape[0] if table.dim() == 2 else table.numel() // _lib.RECORD_BYTES
        if table.device != self.data.device or not table.is_contiguous():
            raise ValueError("record table must be a contiguous tensor on the batch's device")
        if rows < self.nbuf * self.cap:
            raise ValueError(f"record table holds {rows} records, the batch may write {self.nbuf * self.cap}")
        self.recs = table.view(-1)
        self.out.records = table.data_ptr()
        self.out.records_cap = rows

    @property
    def nbytes(self) -> int:
        return self.nbuf * self.buf_len

    def fill_streams(self, first_stream: int, bufs_per_stream: int, seed: int = SYNTH_SEED) -> None:
        """Stream s = first_stream + b // bufs_per_stream holds buffers b (in order)."""
        stream_bytes = bufs_per_stream * self.buf_len
        base = self.data.data_ptr()
        nstreams = (self.nbuf + bufs_per_stream - 1) // bufs_per_stream
        for k in range(nstreams):
            nb = min(bufs_per_stream, self.nbuf - k * bufs_per_stream)
            self.engine.synth_device(base + k * stream_bytes, nb * self.buf_len, seed, first_stream + k, 0,
                                     stream=self.torch.cuda.current_stream().cuda_stream)

    def run(self, buffer_id_base: int = 0, stream: int | None = None) -> None:
        if stream is None:
            stream = self.torch.cuda.current_stream().cuda_stream
        self.engine.run_device(self.data.data_ptr(), self.nbuf, self.buf_len, self.out, stream=stream,
                               buffer_id_base=buffer_id_base)

    def host_results(self):
        """(counts[nbuf], starts[nbuf,cap], lens[nbuf,cap], digests[nbuf,cap,32], total) as numpy."""
        t = self.torch
        t.cuda.synchronize()
        counts = self.counts.cpu().numpy().astype("uint32")
        st = self.starts.view(self.nbuf, self.cap).cpu().numpy().astype("uint32")
        ln = self.lens.view(self.nbuf, self.cap).cpu().numpy().astype("uint32")
        dg = self.digests.view(self.nbuf, self.cap, 32).cpu().numpy()
        return counts, st, ln, dg, int(self.total.item())

    def record_table(self):
        """Dense fingerprint table (total x 48 B) as a device tensor view."""
        n = int(self.total.item())
        return self.recs[: n * _lib.RECORD_BYTES].view(n, _lib.RECORD_BYTES)

    def fill_tar(self, layout: "TarLayout") -> None:
        """Write the tar-like stream of ``layout`` into the batch, piece by piece, with the engine's
        device generator (zero padding by memset); the batch holds stream bytes [0, nbytes)."""
        if layout.total != self.nbytes:
            raise ValueError(f"layout covers {layout.total} bytes, the batch holds {self.nbytes}")
        st = self.torch.cuda.current_stream().cuda_stream
        base = self.data.data_ptr()
        for dst, n, src in layout.pieces:
            if src < 0:
                self.data[dst:dst + n].zero_()
            else:
                self.engine.synth_device(base + dst, n, layout.seed, src, 0, stream=st)


# ---- BASELINE.json configs[4]: the BACKUP_VOLUME archive profile's tar-like stream ----
TAR_SEED = 0x7A5_5DF5
TAR_HEADER_STREAM = 1 << 40  # header of file k = synthetic stream TAR_HEADER_STREAM + k
TAR_BODY_STREAM = 1 << 41    # fresh body of file k = synthetic stream TAR_BODY_STREAM + k


@dataclass
class TarLayout:
    """A tar-like sequential stream ("512-B headers + PRNG file bodies whose
    lengths are log-uniform 1 KiB-64 MiB; 20 % of bodies repeat an earlier body"), as the
    BACKUP_VOLUME profile (VolumeConfigWriter.java:298-307) would receive it from a backup tool.
    Like ustar, every member is a 512-byte header followed by its body zero-padded to a multiple of
    512.  ``pieces`` = (stream offset, length, source stream or -1 for zeros) covering [0, total)
    in order (a source piece is bytes [0, length) of that counter-based synthetic stream);
    ``repeats`` = (copy offset, original offset, length) of every repeated body."""

    total: int
    seed: int
    pieces: list
    bodies: list   # (stream offset, length, source stream) of every body
    repeats: list


def tar_layout(total: int, seed: int = TAR_SEED, repeat_p: float = 0.2, lo_log2: float = 10.0,
               hi_log2: float = 26.0) -> TarLayout:
    import numpy as np

    rng = np.random.default_rng(seed)
    pieces, bodies, repeats = [], [], []
    fresh = []  # indices into bodies of non-repeated bodies
    p = k = 0
    while p < total:
        h = min(512, total - p)
        pieces.append((p, h, TAR_HEADER_STREAM + k))
        p += h
        if p >= total:
            break
        n = int(2.0 ** rng.uniform(lo_log2, hi_log2))
        src = TAR_BODY_STREAM + k
        orig = None
        if fresh and rng.random() < repeat_p:
            orig = bodies[fresh[int(rng.integers(0, len(fresh)))]]
            n, src = orig[1], orig[2]  # the whole earlier body, byte for byte
        n = min(n, total - p)
        pieces.append((p, n, src))
        if orig is not None:
            repeats.append((p, orig[0], n))
        else:
            fresh.append(len(bodies))
        bodies.append((p, n, src))
        p += n
        pad = min((-n) % 512, total - p)
        if pad:
            pieces.append((p, pad, -1))
            p += pad
        k += 1
    return TarLayout(total, seed, pieces, bodies, repeats)
