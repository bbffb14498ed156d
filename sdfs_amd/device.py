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
