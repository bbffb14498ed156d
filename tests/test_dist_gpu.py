"""The pipelined record exchange on the GPU (RCCL, world size 1 on the one-GPU test box): the CUDA
stream/event handling of sdfs_amd.dist.RecordExchange that bench.py runs at N > 1.  World size
2-3 over gloo is covered on CPU by tests/test_dist.py; N = 8 over xGMI is the driver's run."""
import os
import socket

import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_record_exchange_rccl_world1_overlapped_steps():
    import torch
    import torch.distributed as dist

    from sdfs_amd import HipVariableSha256HashEngine
    from sdfs_amd.device import DeviceBatch
    from sdfs_amd.dist import RecordExchange

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        eng = HipVariableSha256HashEngine()
        batch = DeviceBatch(eng, nbuf=64, buf_len=262144)
        ex = RecordExchange(batch.recs.view(-1, 48).shape[0], "cuda:0", depth=2)
        cs = torch.cuda.current_stream()
        want = []
        for step in range(5):  # no host sync between steps: the exchange overlaps the next step
            batch.fill_streams(first_stream=10 * step, bufs_per_stream=8)
            batch.run(buffer_id_base=0, stream=cs.cuda_stream)
            ex.submit(batch.recs.view(-1, 48), batch.total, stream=cs)
            want.append((batch.recs.view(-1, 48).clone(), batch.total.clone()))  # stream-ordered copy
        got = ex.flush()
        torch.cuda.synchronize()
        assert len(got) == 5
        for (g, cl), (wt, wn) in zip(got, want):
            n = int(wn.item())
            assert cl == [n] and n > 0
            assert torch.equal(RecordExchange.compact(g, cl), wt[:n])
        eng.destroy()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_record_exchange_rccl_direct_slots_two_streams():
    """bench.py's production form: two batches in flight on two streams, each engine run writing
    its records straight into the exchange slot it acquired (no snapshot copy)."""
    import torch
    import torch.distributed as dist

    from sdfs_amd import HipVariableSha256HashEngine
    from sdfs_amd.device import DeviceBatch
    from sdfs_amd.dist import RecordExchange

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        eng = HipVariableSha256HashEngine()
        batches = [DeviceBatch(eng, nbuf=64, buf_len=262144) for _ in range(2)]
        ex = RecordExchange(batches[0].recs.view(-1, 48).shape[0], "cuda:0", depth=2, slots=3)
        streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
        for k, b in enumerate(batches):  # different inputs per batch
            b.fill_streams(first_stream=7 * k, bufs_per_stream=8)
        torch.cuda.synchronize()
        refs = []
        for b in batches:  # reference records from each batch's own buffer
            b.run()
            torch.cuda.synchronize()
            refs.append(b.record_table().clone())
        for step in range(6):
            b, s = batches[step & 1], streams[step & 1]
            rec = ex.acquire(stream=s)
            b.set_records(rec)
            b.run(buffer_id_base=0, stream=s.cuda_stream)
            ex.submit(rec, b.total, stream=s)
        got = ex.flush()
        torch.cuda.synchronize()
        assert len(got) == 6
        for step, (g, cl) in enumerate(got):
            want = refs[step & 1]
            assert cl == [want.shape[0]]
            assert torch.equal(RecordExchange.compact(g, cl), want), step
        eng.destroy()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_dedup_index_rccl_world1_matches_local_index():
    import torch
    import torch.distributed as dist

    from sdfs_amd import HipVariableSha256HashEngine
    from sdfs_amd.device import DeviceBatch
    from sdfs_amd.dist import ShardedDedupIndex
    from sdfs_amd.index import HipHashesMap

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        eng = HipVariableSha256HashEngine()
        batch = DeviceBatch(eng, nbuf=64, buf_len=262144)
        batch.fill_streams(first_stream=3, bufs_per_stream=8)
        v = batch.data.view(64, 262144)
        v[32:].copy_(v[:32])  # half the buffers repeat: duplicates across the batch
        batch.run()
        recs = batch.record_table()
        ref_ix, sh_ix = HipHashesMap(1 << 16), HipHashesMap(1 << 16)
        dup_r, loc_r, _, _ = ref_ix.put_records(recs, None, pos_base=5)
        dup_s, loc_s = ShardedDedupIndex(sh_ix).put_records(recs, batch.total, pos_base=5)
        torch.cuda.synchronize()
        n = recs.shape[0]
        assert torch.equal(dup_s, dup_r[:n]) and torch.equal(loc_s, loc_r[:n])
        assert int(dup_s.sum()) >= n // 2
        ref_ix.destroy()
        sh_ix.destroy()
        eng.destroy()
    finally:
        dist.destroy_process_group()
