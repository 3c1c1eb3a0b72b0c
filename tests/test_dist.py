"""Multi-process (world_size 2, gloo, CPU) coverage of bench.py's N>1 path:
sequence sharding is a partition with no data-path exchange, per-rank results
do not depend on the number of ranks, and the timing reduction is a MAX."""
import hashlib
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def queue_get(q, procs, timeout=240):
    """The result a worker puts on q; fails at once when a worker died first."""
    import queue
    import time
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            return q.get(timeout=2)
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f"a worker exited with {dead}"
    raise AssertionError("no result from the workers")


def encode_digest(seed, w=176, h=144, nframes=2):
    """Per-sequence work stand-in: the CPU oracle encoding one short sequence."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    import p64_amd

    frames = [p64_amd.synth_frame(seed, t, w, h) for t in range(nframes)]
    outs = oracle.encode_sequence(frames, w, h, quant=8, me_mode=1, search_limit=31)
    hsh = hashlib.sha256()
    for coef, mb, _, recon in outs:
        hsh.update(coef.tobytes())
        hsh.update(mb.tobytes())
        hsh.update(recon.tobytes())
    return int.from_bytes(hsh.digest()[:7], "little")


def _worker(rank, world, port, streams, q):
    import sys
    sys.path.insert(0, REPO)
    import torch
    import bench

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    seed0, n = bench.shard_seeds(rank, streams)
    digests = torch.tensor([encode_digest(seed0 + k) for k in range(n)], dtype=torch.int64)
    gathered = [torch.zeros_like(digests) for _ in range(world)]
    dist.barrier()
    dist.all_gather(gathered, digests)  # verification only, outside any timed region
    fake_time = 1.0 + rank  # rank 1 is "slower"
    tmax = bench.max_over_ranks(fake_time, world)
    seeds = [bench.shard_seeds(r, streams)[0] + k for r in range(world) for k in range(streams)]
    if rank == 0:
        q.put((torch.cat(gathered).tolist(), tmax, seeds,
               bench.aggregate_rate(world, streams * 99, 10, tmax)))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_matches_single_process():
    world, streams = 2, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, streams, q)) for r in range(world)]
    for p in procs:
        p.start()
    digests, tmax, seeds, rate = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(set(seeds)) == world * streams          # disjoint shards
    assert seeds == list(range(1, 1 + world * streams))  # cover 1..N*S exactly
    single = [encode_digest(s) for s in seeds]
    assert digests == single
    assert tmax == 2.0
    assert np.isclose(rate, world * streams * 99 * 10 / 2.0)


def _root_worker(rank, world, port, S, q):
    """--feed root data path: rank 0 scatters every rank's pictures, each rank
    encodes its shard (CPU oracle as the stand-in), rank 0 gathers the levels."""
    import sys
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import torch

    import bench
    import oracle
    import p64_amd

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    w, h = 176, 144
    pic = w * h * 3 // 2
    all_pics = None
    if rank == 0:
        all_pics = torch.from_numpy(np.stack([p64_amd.synth_frame(1 + i, 0, w, h)
                                              for i in range(world * S)]))
    recv = torch.empty((S, pic), dtype=torch.uint8)
    bench.scatter_pictures(world, rank, all_pics, recv)
    seed0, _ = bench.shard_seeds(rank, S)
    assert all(np.array_equal(recv[k].numpy(), p64_amd.synth_frame(seed0 + k, 0, w, h)) for k in range(S))
    coef = torch.from_numpy(np.stack([
        oracle.encode_frame(w, h, recv[k].numpy(), None, np.zeros(99, np.uint8), intra=True,
                            quant=8)[0] for k in range(S)]))
    bufs = [torch.empty_like(coef) for _ in range(world)] if rank == 0 else None
    bench.gather_outputs(world, rank, coef, bufs)
    if rank == 0:
        q.put(torch.cat(bufs).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_root_feed_scatter_gather():
    import sys
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    import p64_amd

    world, S = 2, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_root_worker, args=(r, world, port, S, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for i in range(world * S):
        exp = oracle.encode_frame(176, 144, p64_amd.synth_frame(1 + i, 0, 176, 144), None,
                                  np.zeros(99, np.uint8), intra=True, quant=8)[0]
        np.testing.assert_array_equal(got[i], exp)


def _bench_json(out: str) -> dict:
    import json
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_launcher_spawns_ranks():
    """`bench.py --gpus 2` with no external launcher starts two ranks itself
    (torch.distributed.run as a child, before any device call); the dry mode
    replaces the GPU step by a host stand-in.  The JSON line reports n_gpus 2,
    the MAX over ranks (rank 1 is slower) and disjoint sequence ranges."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--dry", "--gpus", "2",
                        "--steps", "20", "--streams", "8"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _bench_json(r.stdout)
    assert d["n_gpus"] == 2 and d["dry"] is True
    assert d["seed_ranges"] == [[1, 8], [9, 16]]
    assert d["elapsed_max_s"] >= 20 * 0.002  # rank 1's 2 ms steps bound the MAX
    assert abs(d["value"] - 2 * 8 * 396 * 20 / d["elapsed_max_s"]) < 1e-6 * d["value"]
    # who ran it: the process group's size and one entry per rank (device
    # fields null without a device; on a GPU node each rank's PCI bus id)
    rk = d["ranks"]
    assert rk["world_size"] == 2 and rk["backend"] == "gloo"
    assert [r["rank"] for r in rk["ranks"]] == [0, 1]
    assert [r["local_rank"] for r in rk["ranks"]] == [0, 1]
    assert all(set(r) == {"rank", "local_rank", "host", "pci_bus_id", "device"} for r in rk["ranks"])


def test_bench_n1_launcher_line_shape_matches_plain():
    """The N=1 line under torch.distributed.run (WORLD_SIZE=1 from the
    launcher) has exactly the keys, and ranks block, of a plain N=1 run."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    args = ["--dry", "--gpus", "1", "--steps", "3", "--streams", "4"]
    plain = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args],
                           capture_output=True, text=True, timeout=120, env=env)
    assert plain.returncode == 0, plain.stderr[-2000:]
    launched = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                               "--nproc-per-node=1", "--master-addr=127.0.0.1",
                               f"--master-port={free_port()}", os.path.join(REPO, "bench.py"), *args],
                              capture_output=True, text=True, timeout=240, env=env)
    assert launched.returncode == 0, launched.stderr[-2000:]
    a, b = _bench_json(plain.stdout), _bench_json(launched.stdout)
    assert set(a) == set(b)
    assert set(a["config"]) == set(b["config"])
    for d in (a, b):
        assert d["n_gpus"] == 1 and d["ranks"]["world_size"] == 1
        assert len(d["ranks"]["ranks"]) == 1 and d["ranks"]["distinct_devices"] == 1
        for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                  "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
            assert k in d


def test_bench_refuses_world_mismatch():
    """Under a launcher whose world size differs from --gpus, bench.py exits
    non-zero instead of mislabelling the line."""
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--dry", "--gpus", "2",
                        "--steps", "2"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "refusing" in r.stderr + r.stdout


def _coded_worker(rank, world, port, S, q):
    """--feed root, coded: each rank entropy-codes its shard's pictures (on the
    GPU in bench.py; here the host writer over the CPU oracle's records stands
    in), bench.gather_coded carries the coded bytes + bit counts to rank 0."""
    import sys
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import torch

    import bench
    import oracle
    import p64_amd
    from p64_amd import stream

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    w, h = 176, 144
    seed0, _ = bench.shard_seeds(rank, S)
    streams = [coded_sequence(oracle, p64_amd, stream, seed0 + k, w, h) for k in range(S)]
    stride = max(len(x) for x in streams) + 64 * (rank + 1)  # ranks' buffers differ in size
    out = torch.zeros((S, stride), dtype=torch.uint8)
    for k, x in enumerate(streams):
        out[k, :len(x)] = torch.frombuffer(bytearray(x), dtype=torch.uint8)
    bits = torch.tensor([8 * len(x) for x in streams], dtype=torch.int32)
    got = bench.gather_coded(world, rank, out, bits)
    if rank == 0:
        pays, bl = got
        q.put([bytes(p[i, :int(b[i]) // 8].numpy().tobytes()) for p, b in zip(pays, bl) for i in range(S)])
    else:
        assert got is None
    dist.barrier()
    dist.destroy_process_group()


def coded_sequence(oracle, p64_amd, stream, seed, w, h, n=2):
    """The .p64 of a short closed-loop sequence: the oracle's records through
    the host writer (the GPU coder's bits are byte-identical to it,
    tests/test_gpu_stream.py)."""
    frames = [p64_amd.synth_frame(seed, t, w, h, content=p64_amd.SYNTH_SURVEY) for t in range(n)]
    outs = oracle.encode_sequence(frames, w, h, quant=8, me_mode=1, search_limit=31)
    wr = stream.Writer(stream.format_of(w, h))
    for t, (coef, mb, _, _) in enumerate(outs):
        wr.write_picture(t, mb, coef, 8)
    return wr.end(n)


def test_two_rank_root_feed_gathers_coded_streams():
    """The fed path's coded gather (bench.py --feed root, default --gather
    coded): the streams rank 0 receives from two ranks equal the .p64 bytes a
    single process writes for the same sequences."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    import p64_amd
    from p64_amd import stream

    world, S = 2, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_coded_worker, args=(r, world, port, S, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(got) == world * S
    for i in range(world * S):
        assert got[i] == coded_sequence(oracle, p64_amd, stream, 1 + i, 176, 144), i


def picture_piece(stream, fmt, tr, mb, coef, q, phase):
    """CPU stand-in for the GPU coder's output (p64gpu_vlc_pictures): one
    picture's bits from bit `phase` of byte 0 (the phase bits zero), padded
    to a byte, and the bit count including the phase."""
    wr = stream.Writer(fmt)
    if phase:
        wr.write_bits(b"\0", phase, 0)
    wr.write_picture(tr, mb, coef, q)
    nbits = wr.bits()
    if wr.phase():
        wr.write_bits(b"\0", 8, wr.phase())
    return wr.data(), nbits


def _pieces_worker(rank, world, port, S, n, q):
    """--feed root, coded, as bench.py runs it: every step each rank codes
    its sequences' next picture at each sequence's running bit phase and
    gathers the pieces to rank 0 (bench.gather_coded, sized by the MAX
    all-reduce of the longest piece); rank 0 stitches them per sequence
    (bench.stitch_pieces)."""
    import sys
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import torch

    import bench
    import oracle
    import p64_amd
    from p64_amd import stream

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    w, h = 176, 144
    fmt = stream.format_of(w, h)
    seed0, _ = bench.shard_seeds(rank, S)
    recs = []
    for k in range(S):
        frames = [p64_amd.synth_frame(seed0 + k, t, w, h, content=p64_amd.SYNTH_SURVEY) for t in range(n)]
        recs.append(oracle.encode_sequence(frames, w, h, quant=8, me_mode=1, search_limit=31))
    seq_bits = [0] * S
    writers = {g: stream.Writer(fmt) for g in range(world * S)} if rank == 0 else None
    stride = 16384 + 64 * rank  # (ranks' buffers differ in size)
    for t in range(n):
        out = torch.zeros((S, stride), dtype=torch.uint8)
        bits = torch.zeros(S, dtype=torch.int32)
        for k in range(S):
            coef, mb, _, _ = recs[k][t]
            data, nb = picture_piece(stream, fmt, t % 32, mb, coef, 8, seq_bits[k] & 7)
            out[k, :len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
            bits[k] = nb
            seq_bits[k] += nb - (seq_bits[k] & 7)
        mx = bits.to(torch.int64).max().reshape(1) if t % 2 else None  # (both ways to the size)
        got = bench.gather_coded(world, rank, out, bits, mx=mx)
        if rank == 0:
            pays, bls = got
            pieces = {r * S + i: pays[r][i].numpy().tobytes() for r in range(world) for i in range(S)}
            nbits = {r * S + i: int(bls[r][i]) for r in range(world) for i in range(S)}
            bench.stitch_pieces(writers, pieces, nbits)
        else:
            assert got is None
    if rank == 0:
        q.put([writers[g].end(n % 32) for g in range(world * S)])
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_root_feed_stitches_per_picture_pieces():
    """The fed path's per-picture pieces, each coded at its sequence's bit
    phase, gathered step by step from two ranks and stitched on rank 0 equal
    the .p64 a single process writes for the same sequences (p64.c:524-613,
    stream.c:142-150)."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    import p64_amd
    from p64_amd import stream

    world, S, n = 2, 2, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_pieces_worker, args=(r, world, port, S, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = queue_get(q, procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(got) == world * S
    for i in range(world * S):
        assert got[i] == coded_sequence(oracle, p64_amd, stream, 1 + i, 176, 144, n=n), i
