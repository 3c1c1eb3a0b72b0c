#!/usr/bin/env python3
"""bench.py -- macroblocks/s of the MI355X encode hot path (BASELINE.json).

Configs (BASELINE.json `configs`; `--config`):
  inter   (default; configs[2], the metric's config) CIF 352x288 inter pictures,
          brute-force FastBME at SearchLimit 31 ([-15,14]^2, 900 candidates,
          me.c:206) + MTYPE decision + prediction/loop filter + ChenDct +
          quantisation + zigzag + CBP + IQ/ChenIDct reconstruction: two
          launches per step, k_motion<2> (the search, one wave per MB) and
          k_inter_mbg (the rest, one lane per 8x8 block); `--mode tss` for the
          shipped StepBME.
  intra   (configs[1]) CIF intra pictures: ChenDct + FlatQuant + zigzag + IQ/IDCT
          reconstruction (k_intra_mbg).  HBM-bound.
  decode  (configs[4]) decoder reconstruction (k_recon_mbg) of a CIF stream the
          GPU encoder produced (FULL search, q=8): IZigzag + IQ + ChenIDct +
          prediction/loop filter.  HBM-bound.
  4cif    (configs[3]) 704x576 inter, FULL SL=31; with N>1 use `--feed root`
          (rank 0 RCCL-scatters pictures and gathers levels every step).

Each GPU encodes S independent closed-loop sequences (the chunks `p64 -a first
-b last` would encode); one STEP = one picture of every
sequence = ONE launch over S*nmb macroblocks.  W warmup steps run untimed, K
steps are timed with inputs resident in HBM (a distinct input picture per step
up to 256 slots), after a steady-state spin-up: the same K launches into
scratch outputs, replayed for --spinup-ms (timed_region).  The default `inter` run also measures the intra and decode
configs on the same pictures and reports them under "configs" (each with its own
roofline), so one driver run carries all three kernels.

`--content` picks the input: survey (default: SURVEY.md 8(d)'s content --
128 + 50 sin(x/7) cos(y/11) + 30 sin((x+y)/23) + N(0,12) texture translated by
(+3,-2) px per picture + N(0,4) temporal noise, seeds 1..S), synth (the
builder's value-noise generator: per-seed motion, weaker temporal noise,
scene-cut / noise-free / low-contrast seed classes), pan15 (texture panned
+-15 px per picture: the search range edge), noise (uniform random bytes:
nothing prunes) or flat (constant planes: SAD ties everywhere) -- the stress
sets of SURVEY.md 8(d).

Multi-GPU: `--gpus N` without a launcher starts N ranks itself (torch
distributed run as a child process, before any GPU call); under a launcher
WORLD_SIZE must equal --gpus.  One process per GPU, RCCL; weak scaling.  The
timed region is bracketed by barrier + synchronize; the MAX over ranks is
reported.  `--dry` replaces the GPU work by a host stand-in (gloo, no device)
to test the launcher and the reductions on a CPU box.

Extra objects on the JSON line: roofline (HBM, algorithmic bytes),
roofline_sad (FULL: exhaustive-search equivalent), cpu_baseline (the reference
encoder from oracle/_ref, 1 process and one per core of the box's share).
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "macroblocks/s (full-search ME+DCT+quant), CIF inter; % HBM roofline"
METRICS = {
    "inter": METRIC,
    "4cif": "macroblocks/s (full-search ME+DCT+quant), 4CIF inter; % HBM roofline",
    "intra": "macroblocks/s (ChenDct+quant+zigzag+recon), CIF intra; % HBM roofline",
    "decode": "macroblocks/s (IQ+ChenIDct+prediction+recon), CIF decode; % HBM roofline",
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
# v_sad_u8 = 4 byte-absolute-differences per lane.  It issues at HALF rate on
# gfx950 (tools/ubench_sad.hip: 0.57e12 wave-instr/s chip-wide = 4 cycles per
# wave64 instruction per SIMD), so the ceiling is 256 CUs x 4 SIMDs x 16 lanes
# per clock x 4 B x 2.4 GHz (MI355X_MICROARCH.md chip table).
SAD_PEAK = 256 * 4 * 16 * 4 * 2.4e9
# algorithmic HBM bytes per macroblock:
#   inter: read cur 384 + previous recon 384 + last_intra 1;
#          write recon 384 + p64_mb_rec 4 + p64_me_rec 28 + last_intra 1 +
#          nonzero-block mask 1, and
#          128 per transmitted block (MTYPE with coefficients, CBP bit set:
#          counted from the last step's records, coded_level_bytes; the kernel
#          writes every block with a nonzero level, include/p64gpu.h)
#   intra: read cur 384; write levels 768 + recon 384 + p64_mb_rec 4 + last_intra 1
#   decode: per MB record 4 + UseQuant 1 + coded flag 1, 128 per coded block,
#          384 prediction source if not intra, 384 recon write (counted exactly
#          from the records of each launch, see decode_bytes)
BYTES_PER_MB_FIXED = 384 + 384 + 1 + 384 + 4 + 28 + 1 + 1
READ_BYTES_PER_MB = 384 + 384 + 1
INTRA_BYTES_PER_MB = 384 + 768 + 384 + 4 + 1
# per-kernel means over the timed region of the driver's command (rocprofv3
# --kernel-trace of `bench.py --steps 20 --warmup 5 --no-cpu`, reduced by
# tools/timed_region.py --json; the spin-up's replays are outside the region)
PROFILE_TIMED = "profiles/r06_timed_region.json"  # {workload key: {kernel: mean us}}
# executed v_sad_u8 work of k_motion per launch (tools/sad_count.py side build)
PROFILE_SAD = "profiles/sad_executed.json"
VALU_BUSY_NOTE = ("derived, not a busy counter: SQ_INSTS_VALU (PMC) x the kernel's mean VALU issue cost "
                  "(static ISA mix priced by tools/ubench_valu's measured clocks, tools/pmc_merge.py) / "
                  "(1024 SIMDs x kernel cycles)")
MAX_SLOTS = 256  # distinct input pictures per sequence kept resident (~10 GB at S=256 CIF)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", choices=("inter", "intra", "decode", "4cif"), default="inter")
    p.add_argument("--mode", choices=("full", "tss"), default="full")
    p.add_argument("--content", choices=("survey", "synth", "pan15", "noise", "flat"), default="survey")
    p.add_argument("--search-limit", type=int, default=31)
    p.add_argument("--quant", type=int, default=8)
    p.add_argument("--width", type=int, default=None)
    p.add_argument("--height", type=int, default=None)
    p.add_argument("--streams", type=int, default=None, help="sequences per GPU")
    p.add_argument("--no-extra", action="store_true",
                   help="inter: skip the intra/decode measurements under 'configs'")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    p.add_argument("--cpu-procs", type=int, default=None,
                   help="processes of the multi-core CPU leg (default: this box's CPU share)")
    p.add_argument("--cpu-frames", type=int, default=300,
                   help="pictures per CPU process (300 CIF pictures: a few s of CPU work)")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--no-vlc", action="store_true", help="skip the encode+entropy-coding measurement")
    p.add_argument("--feed", choices=("local", "root"), default="local",
                   help="local: every rank generates its own sequences (default, no data-path "
                        "collective); root: rank 0 holds all inputs, RCCL-scatters each step's "
                        "pictures and gathers the levels/records back (the timed step includes both)")
    p.add_argument("--gather", choices=("coded", "levels"), default="coded",
                   help="--feed root: what rank 0 collects each step -- coded (default: every "
                        "picture's H.261 bits, entropy-coded on its rank's GPU inside the step) or "
                        "levels (the int16 levels + records, 768 B/MB: parity debugging)")
    p.add_argument("--eager", action="store_true",
                   help="launch every timed step from Python instead of replaying a captured HIP graph")
    p.add_argument("--spinup-ms", type=int, default=150,
                   help="steady state before each timed region: the same K launches on scratch "
                        "outputs, replayed back to back for at least this long (the chip ramps "
                        "its clocks over tens of ms of load); 0 = off")
    p.add_argument("--dry", action="store_true",
                   help="no device: gloo + a host stand-in step (launcher/reduction tests)")
    p.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    a = p.parse_args(argv)
    big = a.config == "4cif"
    a.width = a.width or (704 if big else 352)
    a.height = a.height or (576 if big else 288)
    a.streams = a.streams or (64 if big else 256)
    if a.steps < 1 or a.warmup < 0:
        p.error("--steps must be >= 1 and --warmup >= 0")
    return a


def shard_seeds(rank: int, streams: int) -> tuple[int, int]:
    """Weak scaling: rank r owns sequences seed0 .. seed0+streams-1."""
    return 1 + rank * streams, streams


def max_over_ranks(value: float, world: int, device=None) -> float:
    """MAX of a per-rank float over the process group (identity at world 1)."""
    if world == 1:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_ranks_ok(ok: bool, world: int, device=None) -> bool:
    """True iff every rank passed (MIN over ranks of a 0/1 flag)."""
    if world == 1:
        return ok
    import torch
    import torch.distributed as dist

    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def aggregate_rate(world: int, units_per_rank_step: int, steps: int, tmax: float) -> float:
    """Whole-job throughput: every rank's units over the slowest rank's time."""
    return world * units_per_rank_step * steps / tmax


def scatter_pictures(world: int, rank: int, all_pics, recv):
    """--feed root: rank 0 holds [world*S, pic] bytes; rank r receives rows
    r*S..(r+1)*S-1 (its shard_seeds range) into recv [S, pic]."""
    import torch.distributed as dist
    if world == 1:
        recv.copy_(all_pics)
        return recv
    chunks = list(all_pics.chunk(world)) if rank == 0 else None
    dist.scatter(recv, scatter_list=chunks, src=0)
    return recv


def gather_outputs(world: int, rank: int, local, bufs):
    """--feed root: every rank's output tensor is collected on rank 0 (bufs,
    one per rank, rank 0 only)."""
    import torch
    import torch.distributed as dist
    if world == 1:
        if bufs is not None:
            bufs[0].copy_(local)
        return bufs
    # as bytes: int16 levels are not an RCCL/NCCL (nor gloo) element type
    byte = lambda t: t.contiguous().view(torch.uint8)  # noqa: E731
    dist.gather(byte(local), gather_list=[byte(b) for b in bufs] if rank == 0 else None, dst=0)
    return bufs


def gather_coded(world, rank, out, bits, mx=None):
    """--feed root, coded: every rank's entropy-coded pictures to rank 0.
    out [S, stride] uint8 holds each picture's bits from byte 0 (at its
    sequence's bit phase), bits [S] int32 their counts incl. the phase.  One
    MAX all-reduce of the longest picture (mx: a [1] int64 tensor holding
    this rank's longest, else computed here), then the first nb bytes of
    every picture (nb = that length, 4-aligned) and the counts, gathered as
    bytes: ~S x nb bytes per rank instead of S x nmb x 772 for the levels.
    The size is read back with .item() on the CURRENT stream (CodedFeed runs
    this on a side stream, so the encode stream does not wait).  Returns on
    rank 0 ([world] payloads [S, nb], [world] bit counts [S]), else None."""
    import torch
    import torch.distributed as dist
    if mx is None:
        mx = bits.to(torch.int64).max().reshape(1)
    if world > 1:
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    nb = (int(mx.item()) + 7) // 8
    nb = max(4, (nb + 3) // 4 * 4)
    payload = out[:, :nb].contiguous()
    b32 = bits.to(torch.int32).contiguous()
    if world == 1:
        return [payload], [b32]
    pays = [torch.empty_like(payload) for _ in range(world)] if rank == 0 else None
    bl = [torch.empty_like(b32) for _ in range(world)] if rank == 0 else None
    dist.gather(payload, gather_list=pays, dst=0)
    dist.gather(b32.view(torch.uint8), gather_list=[b.view(torch.uint8) for b in bl] if rank == 0 else None,
                dst=0)
    return (pays, bl) if rank == 0 else None


def stitch_pieces(writers, pieces, bits):
    """Rank 0: appends one step's coded pictures to their sequences' streams.
    writers: {sequence: stream.Writer}; pieces[sequence] the picture's bytes
    from byte 0, coded at the writer's bit phase (its first byte shares the
    stream's pending byte), bits[sequence] its bit count incl. that phase
    (p64s_write_bits: the pending byte ORed, the rest appended; the writer
    closes the stream with p64s_write_end's padding, stream.c:142-150)."""
    for s, wr in writers.items():
        b = int(bits[s])
        if b == 0xFFFFFFFF or b < 0:
            raise RuntimeError(f"coded picture of sequence {s}: invalid record or overflow")
        wr.write_bits(pieces[s], b, wr.phase())


class CodedFeed:
    """--feed root --gather coded: the rank's pictures entropy-coded on its
    GPU each step, every picture at its sequence's running bit phase
    (p64gpu_vlc_pictures with seq_bits / max_bits: the coder continues each
    sequence's stream on the device; p64EncodeSequence's continuous stream,
    p64.c:524-613), and the coded pictures gathered to rank 0 on a side
    stream.  Forked (the default): step t's coder runs on the side stream
    behind an event on the encode stream, beside step t+1's encode; the
    encode outputs alternate between two sets, and before_encode(t) makes the
    encode stream wait for the coder that read its set (step t-2's).  At N>1
    the gather of step t-1 (a MAX all-reduce of the longest picture, its size
    read back on the side stream, then the payloads) is issued before step
    t's coder, so the host's only wait ends with step t-1's coder and the
    encode stream never waits for the host; at one rank the gather is the
    identity and follows each coder at once (no size read back).  finish()
    gathers the last step.  (P64_FEED_FORK=0: the coder on the encode
    stream, the gather one step late -- round 6's first form.)
    Rank 0 keeps the pieces of the sequences in `keep` (global indices) for
    stitch_pieces; verification happens after the timed region."""

    def __init__(self, torch, p64s, world, rank, S, w, h, quant, keep=()):
        import torch.distributed as dist
        self.torch, self.p64s, self.dist = torch, p64s, dist
        self.world, self.rank, self.S, self.w, self.h = world, rank, S, w, h
        nmb = (w // 16) * (h // 16)
        self.bufs = [p64s.vlc_buffers(S, w, h) for _ in range(2)]
        self.gq = torch.full((S, nmb // 33), quant, dtype=torch.uint8, device="cuda")
        self.trs = [torch.full((S,), t, dtype=torch.int32, device="cuda") for t in range(32)]
        self.seq_bits = torch.zeros(S, dtype=torch.int64, device="cuda")  # bits so far per sequence
        self.mx = [torch.zeros(1, dtype=torch.int32, device="cuda") for _ in range(2)]  # the longest picture
        self.bits = [None, None]
        self.ev = [torch.cuda.Event(), torch.cuda.Event()]  # step t's coder done (t % 2)
        self.enc_ev = [torch.cuda.Event(), torch.cuda.Event()]  # step t's encode done (forked coder)
        # (P64_FEED_SIDE=0: gathers on the encode stream itself -- diagnostic)
        self.side = torch.cuda.Stream() if os.environ.get("P64_FEED_SIDE", "1") != "0" else torch.cuda.current_stream()
        # the coder on the side stream, beside the next step's encode (the
        # encode's outputs alternate between two sets, see before_encode)
        self.fork = os.environ.get("P64_FEED_FORK", "1") != "0" and self.side != torch.cuda.current_stream()
        self.pending = None
        # rank 0: (rank, local row) of each kept global sequence
        self.keep = {g: (g // S, g % S) for g in keep if g < world * S}
        rows = {}
        for g, (r, i) in sorted(self.keep.items()):
            rows.setdefault(r, ([], []))
            rows[r][0].append(g)
            rows[r][1].append(i)
        self.keep_rows = {r: (gs, torch.tensor(ix, dtype=torch.int64, device="cuda")) for r, (gs, ix) in rows.items()}
        self.kept = []  # per coded step: {global sequence: (piece tensor, bits tensor)}
        self.steps = []

    def before_encode(self, t):
        """Forked coder: step t's encode overwrites the output set step t-2's
        coder reads (the sets alternate), so the encode stream waits for that
        coder's event first (it ended during step t-1's encode)."""
        if self.fork:
            self.torch.cuda.current_stream().wait_event(self.ev[t % 2])

    def code(self, t, o, vlc=None):
        """Step t's pictures (outputs o of the encode) into bits, then the
        gather of step t-1.  Forked (the default): the gather of step t-1 is
        issued first on the side stream, then step t's coder behind an event
        on the encode stream, so the coder of step t runs beside the encode
        of step t+1 and the host's one wait (the gather's size read-back)
        ends when step t-1's coder does.  Otherwise (P64_FEED_FORK=0) the
        coder runs on the encode stream (code_gpu + code_host).
        vlc: a prepared coder launch (stream.prepare_vlc on the side stream)
        and its bits, instead of code_gpu's call."""
        torch = self.torch
        if not self.fork:
            torch.cuda.current_stream().wait_stream(self.side)  # (the gather of step t-2 has read buffer t % 2)
            if vlc is None:
                self.code_gpu(t, o)
            else:
                vlc[0]()
                self.bits[t % 2] = vlc[1]
            self.code_host(t)
            return
        self.enc_ev[t % 2].record(torch.cuda.current_stream())
        if self.pending is not None:
            self._gather(self.pending)
            self.pending = None
        with torch.cuda.stream(self.side):
            self.side.wait_event(self.enc_ev[t % 2])
            if vlc is None:
                self.code_gpu(t, o)
            else:
                vlc[0]()
                self.bits[t % 2] = vlc[1]
            self.ev[t % 2].record(self.side)
        if self.world == 1:
            # no size read-back at one rank, so step t's gather follows its
            # coder at once: issued before it (one step late), its small
            # kernels waited ~90 us for the CUs the encode held and delayed
            # the coder behind them (profiles/r06n_fed_trace.txt)
            self._gather(t)
        else:
            self.pending = t

    def code_gpu(self, t, o):
        """The device work of step t's coding on the current stream (no host
        synchronisation, capturable in a HIP graph): the coder, which takes
        each picture's bit phase from its sequence's running bit count,
        advances it and keeps the step's longest picture (p64gpu_vlc_args
        seq_bits / max_bits, ABI v3: two launches, no bookkeeping kernels).
        The caller has made the stream wait for the side stream first."""
        k = t % 2
        _, bits = self.p64s.vlc_pictures(o.mb, o.coef, self.gq, self.trs[t % 32], width=self.w, height=self.h,
                                         buffers=self.bufs[k], host_bits=False, blk_bits=o.vlc_bits,
                                         seq_bits=self.seq_bits, max_bits=self.mx[k])
        self.bits[k] = bits

    def code_host(self, t):
        """After step t's device work is issued: its event, and the gather of
        step t-1 on the side stream."""
        self.ev[t % 2].record(self.torch.cuda.current_stream())
        if self.pending is not None:
            self._gather(self.pending)
        self.pending = t

    def finish(self):
        if self.pending is not None:
            self._gather(self.pending)
            self.pending = None
        self.torch.cuda.current_stream().wait_stream(self.side)

    def _gather(self, t):
        torch = self.torch
        k = t % 2
        with torch.cuda.stream(self.side):
            self.side.wait_event(self.ev[k])
            if self.world == 1:
                # one rank: its pictures are already resident on rank 0 (the
                # gather is the identity), so no size is read back -- the kept
                # pieces below are whole buffer rows
                got = ([self.bufs[k][0]], [self.bits[k]])
            else:
                got = gather_coded(self.world, self.rank, self.bufs[k][0], self.bits[k], mx=self.mx[k])
            if got is not None and self.keep:
                pays, bls = got
                # one indexing op per rank for the kept sequences' pieces
                self.kept.append([(gs, pays[r].index_select(0, ix), bls[r].index_select(0, ix))
                                  for r, (gs, ix) in self.keep_rows.items()])
                self.steps.append(t)

    def streams(self, fmt, end_tr):
        """Rank 0, after the run: the kept sequences' stitched .p64 streams
        ({global sequence: bytes}, closed like p64seq_finish) and bit counts."""
        self.torch.cuda.synchronize()
        writers = {g: self.p64s.Writer(fmt) for g in self.keep}
        for t, per in zip(self.steps, self.kept):
            pieces, bits = {}, {}
            for gs, pay, bl in per:
                pay, bl = pay.cpu().numpy(), bl.cpu().numpy()
                for j, g in enumerate(gs):
                    pieces[g] = pay[j].tobytes()
                    bits[g] = int(bl[j]) & 0xFFFFFFFF
            if os.environ.get("P64_FEED_SYNC", "0") != "0":  # (diagnostic)
                print(f"kept step {t}: " + " ".join(f"{g}:{bits[g]}" for g in sorted(bits)),
                      file=sys.stderr, flush=True)
            stitch_pieces(writers, pieces, bits)
        out = {}
        for g, wr in writers.items():
            nbits = wr.bits()
            out[g] = (wr.end(end_tr), nbits)
        return out


def verify_coded(args, p64_amd, p64s, src, slot, streams, upto, w, h, mode):
    """The stitched streams of --feed root against the host writer over the
    CPU oracle's records of the same sequences (closed loop, pictures
    0..upto at TR t % 32, GQUANT = the run's q, closed like p64seq_finish):
    byte-identical .p64 (what the GPU coder writes equals p64s_write_picture,
    tests/test_gpu_stream.py; p64.c:524-613, stream.c:142-150)."""
    import hashlib
    import oracle
    from concurrent.futures import ThreadPoolExecutor
    oracle.lib()
    fmt = p64s.format_of(w, h)

    def one(g):
        fr = [src[slot(t), g].cpu().numpy() for t in range(upto + 1)]
        outs = oracle.encode_sequence(fr, w, h, quant=args.quant, me_mode=mode, search_limit=args.search_limit)
        wr = p64s.Writer(fmt)
        for t, (coef, mb, _, _) in enumerate(outs):
            wr.write_picture(t % 32, mb, coef, args.quant)
        return g, wr.end((upto + 1) % 32)

    with ThreadPoolExecutor(max(1, len(streams))) as ex:
        want = dict(ex.map(one, sorted(streams)))
    res = {f"seq{1 + g}": {"ok": streams[g][0] == want[g], "bytes": len(streams[g][0]),
                           "sha256": hashlib.sha256(streams[g][0]).hexdigest()[:16]} for g in sorted(streams)}
    return {"ok": all(r["ok"] for r in res.values()), "pictures": upto + 1, "sequences": res,
            "note": "rank 0 stitched each checked sequence's gathered per-picture pieces (every rank's "
                    "first sequence and rank 0's checked ones) into its .p64 (p64s_write_bits at the "
                    "stream's phase, closed by p64s_write_end): equal to the host writer over the "
                    "CPU oracle's records of the same pictures"}


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv) -> int:
    """--gpus N without a launcher: run N ranks under torch.distributed.run as a
    CHILD process (nothing here has touched the GPU) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def rank_info(world, rank, local, dist, torch=None):
    """Who ran the line: the world size torch.distributed sees,
    each rank's device as the HIP runtime names it (PCI domain:bus:device --
    N ranks on N distinct devices show N distinct ids) and the RCCL version
    (torch.cuda.nccl, the library backend "nccl" loads).  Without a device
    (--dry) the device fields are null.  Collective: every rank calls it."""
    me = {"rank": rank, "local_rank": local, "host": socket.gethostname(), "pci_bus_id": None,
          "device": None}
    rccl = None
    if torch is not None:
        p = torch.cuda.get_device_properties(local)
        me["pci_bus_id"] = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
        me["device"] = p.name
        rccl = ".".join(str(v) for v in torch.cuda.nccl.version())
    if world > 1:
        every = [None] * world
        dist.all_gather_object(every, me)
    else:
        every = [me]
    return {"world_size": dist.get_world_size() if world > 1 else 1,
            "backend": dist.get_backend() if world > 1 else None,
            "rccl_version": rccl, "ranks": every,
            "distinct_devices": len({(r["host"], r["pci_bus_id"]) for r in every})}


def box_cores() -> int:
    """CPU share of this process (the GPU box exports OMP_NUM_THREADS = its share;
    os.cpu_count() there counts the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


# ---------------------------------------------------------------------------
# CPU baseline (rank 0, N = 1 only; runs before the GPU is touched)

def write_y4m(path, frames, w, h):
    with open(path, "wb") as f:
        f.write(b"YUV4MPEG2 W%d H%d F30000:1001 Ip A0:0 C420jpeg\n" % (w, h))
        for fr in frames:
            f.write(b"FRAME\n")
            f.write(fr.tobytes())


def _cpu_procs(cmds, env, stdin_path=None):
    """Run the commands as concurrent processes; wall seconds."""
    t0 = time.perf_counter()
    ins = [open(stdin_path) if stdin_path else subprocess.DEVNULL for _ in cmds]
    ps = [subprocess.Popen(c, env=env, stdin=i, stdout=subprocess.DEVNULL) for c, i in zip(cmds, ins)]
    rc = [p.wait() for p in ps]
    dt = time.perf_counter() - t0
    for i in ins:
        if stdin_path:
            i.close()
    if any(rc):
        raise RuntimeError(f"reference run failed: {rc}")
    return dt


def _cpu_leg(run, nprocs, units_per_proc, sample, extra=""):
    """One CPU-baseline leg: `run(k)` -> wall seconds of k concurrent processes,
    first 1 process, then nprocs (this box's CPU share)."""
    dt1 = run(1)
    dtn = run(nprocs) if nprocs > 1 else dt1
    return {"value": round(nprocs * units_per_proc / dtn, 1), "unit": "macroblocks/s", "cores": nprocs,
            "kind": "reference",
            "single_process": {"value": round(units_per_proc / dt1, 1), "cores": 1, "seconds": round(dt1, 2)},
            "sample": f"{sample}; {nprocs} concurrent processes (this box's CPU share), "
                      f"{nprocs * units_per_proc} MBs in {dtn:.2f} s wall; single_process: "
                      f"{units_per_proc} MBs in {dt1:.2f} s{extra}"}


def cpu_baselines(args, legs):
    """The reference itself (oracle/_ref: the unmodified reference objects;
    p64hook adds only the link-time wraps of oracle/ref_hooks.c), timed on this
    box's host cores before the GPU is touched, per leg:
      inter   the encoder on y4m files of the same generator (FastBME SL via
              P64REF_ME=full, or the shipped StepBME for --mode tss)
      intra   the encoder under `-o` with program tests/golden/progs/intra_only
              (MTYPE 0 everywhere, p64.c:761-768) and P64REF_ME=none (no search:
              the records are unused), i.e. ChenDct + quantisation + VLC + IQ/IDCT
      decode  `p64 -d` (p64DecodeSequence p64.c:1022) of the reference's own
              encoding of those files, y4m output
    Returns {leg: cpu_baseline object}; a leg without a reference path (4CIF:
    p64.c:1477-1520 and me.c:49-58 stop at CIF) times the clean-room port."""
    import p64_amd  # host-only synth (no GPU use)

    w, h = args.width, args.height
    fmt = {(352, 288): "-CIF", (176, 144): "-QCIF", (352, 240): "-NTSC"}.get((w, h))
    nmb = (w // 16) * (h // 16)
    cores = box_cores()
    procs = max(1, min(args.cpu_procs or cores, cores))
    nfr = args.cpu_frames
    hook = os.path.join(REPO, "oracle", "_ref", "p64hook")
    out = {}
    if not fmt or not os.access(hook, os.X_OK):
        return {leg: cpu_port(args, p64_amd, w, h, nmb) for leg in legs if leg in ("inter", "4cif")}
    with tempfile.TemporaryDirectory() as td:
        for k in range(procs):
            write_y4m(os.path.join(td, f"s{k}.y4m"), host_frames(p64_amd, args.content, 1 + k, nfr, w, h), w, h)
        env = dict(os.environ)
        env.pop("P64REF_DUMP", None)

        def enc_cmds(n, extra=()):
            return [[hook, fmt, "-y4m", "-a", "0", "-b", str(nfr - 1), "-q", str(args.quant),
                     "-i", str(args.search_limit), *extra, os.path.join(td, f"s{k}"), "-z", ".y4m",
                     "-s", os.path.join(td, f"s{k}.p64")] for k in range(n)]
        desc = (f"{nfr}-picture {w}x{h} y4m sequence per process (content {args.content}, host "
                f"generator{'' if args.content in ('survey', 'synth') else ' of the same kind'}), "
                f"q={args.quant}")
        if "inter" in legs or "decode" in legs:
            me = "FastBME SL=%d" % args.search_limit if args.mode == "full" else "StepBME (TSS)"
            env_i = dict(env, P64REF_ME="full") if args.mode == "full" else env
            leg = _cpu_leg(lambda n: _cpu_procs(enc_cmds(n), env_i), procs, nfr * nmb,
                           f"reference encoder (oracle/_ref/p64hook, {me}), {desc} (first picture intra)",
                           "; includes the reference's VLC and file I/O (compare with_vlc)")
            if "inter" in legs:
                out["inter"] = leg
        if "decode" in legs:  # the streams the inter leg wrote (s0..s{procs-1}.p64)
            def dec_cmds(n):
                return [[hook, "-d", "-y4m", "-s", os.path.join(td, f"s{k}.p64"),
                         os.path.join(td, f"d{k}")] for k in range(n)]
            out["decode"] = _cpu_leg(lambda n: _cpu_procs(dec_cmds(n), env), procs, nfr * nmb,
                                     f"reference decoder (p64 -d, p64DecodeSequence p64.c:1022) of the "
                                     f"reference's own encoding ({args.mode.upper()}) of a {desc}, "
                                     f"y4m output", "; includes VLC parsing and file I/O")
        if "intra" in legs:
            prog = os.path.join(REPO, "tests", "golden", "progs", "intra_only.prog")
            env_n = dict(env, P64REF_ME="none")
            out["intra"] = _cpu_leg(lambda n: _cpu_procs(enc_cmds(n, ("-o",)), env_n, prog), procs,
                                    nfr * nmb,
                                    f"reference encoder under -o intra_only.prog (every MB MTYPE 0, "
                                    f"p64.c:761-768) with the search hooked out (P64REF_ME=none), {desc}",
                                    "; includes the interpreter call per MB, VLC and file I/O")
    return out


def host_frames(p64_amd, content, seed, n, w, h):
    """Host pictures for the CPU legs: the survey or synth generator (the same
    bytes as the device one), or the stress contents of make_inputs in kind -- uniform noise,
    one constant per sequence, picture 0 panned by +-15 px per picture with
    +-3 noise (numpy, seeded; the device versions draw from torch's generator)."""
    import numpy as np
    if content in p64_amd.CONTENTS:
        return [p64_amd.synth_frame(seed, t, w, h, content=p64_amd.CONTENTS[content]) for t in range(n)]
    pic = w * h * 3 // 2
    rng = np.random.default_rng(1000 + seed)
    if content == "noise":
        return [rng.integers(0, 256, pic, dtype=np.uint8) for _ in range(n)]
    if content == "flat":
        return [np.full(pic, (seed * 37 + 1) % 224 + 16, np.uint8) for _ in range(n)]
    base = p64_amd.synth_frame(seed, 0, w, h)
    vx, vy = (15 if seed % 2 == 0 else -15), (15 if (seed // 2) % 2 == 0 else -15)
    planes = ((0, w, h, 1), (w * h, w // 2, h // 2, 2), (w * h + w * h // 4, w // 2, h // 2, 2))
    out = []
    for t in range(n):
        f = np.empty(pic, np.uint8)
        for off, pw, ph, div in planes:
            src = base[off:off + pw * ph].reshape(ph, pw).astype(np.int16)
            moved = np.roll(src, (t * vy // div, t * vx // div), (0, 1))
            f[off:off + pw * ph] = (moved + rng.integers(-3, 4, moved.shape)).clip(0, 255).reshape(-1)
        out.append(f)
    return out


def cpu_port(args, p64_amd, w, h, nmb):
    """The clean-room port (scalar, one core) where the reference has no path."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle

    n = min(args.cpu_frames, 12 if nmb <= 396 else 4)
    frames = host_frames(p64_amd, args.content, 1, n, w, h)
    t0 = time.perf_counter()
    oracle.encode_sequence(frames, w, h, quant=args.quant, me_mode=1 if args.mode == "full" else 0,
                           search_limit=args.search_limit)
    dt = time.perf_counter() - t0
    mbs = len(frames) * nmb
    note = ("no reference path: the reference cannot encode 4CIF (p64.c:1477-1520 formats; "
            "me.c:49-58 records sized for CIF), so the clean-room port stands in; "
            if (w, h) == (704, 576) else "")
    return {"value": round(mbs / dt, 1), "unit": "macroblocks/s", "cores": 1, "kind": "port",
            "single_process": {"value": round(mbs / dt, 1), "cores": 1, "seconds": round(dt, 2)},
            "sample": f"{note}oracle/p64_oracle.c (scalar, exhaustive search, no early exit) on "
                      f"{len(frames)} pictures of one {w}x{h} sequence; {mbs} MBs in {dt:.2f} s"}


# ---------------------------------------------------------------------------
# inputs

def make_inputs(torch, p64_amd, content, w, h, seed0, S, nslots):
    """[nslots][S][picture] uint8 on the device.  survey / synth: the seeded
    integer generators (same bytes as the host ones the CPU legs use); the stress sets are
    generated on the device with torch (seeded): pan15 = picture 0 of the synth
    sequence translated by (+-15, +-15) px per picture (wrapping), plus
    uniform +-3 noise; noise = uniform bytes; flat = one constant per sequence."""
    pic = w * h * 3 // 2
    if content in p64_amd.CONTENTS:
        return p64_amd.synth_frames_device(w, h, seed0, S, 0, nslots, content=p64_amd.CONTENTS[content])
    g = torch.Generator(device="cuda")
    g.manual_seed(1000 + seed0)
    if content == "noise":
        return torch.randint(0, 256, (nslots, S, pic), dtype=torch.uint8, device="cuda", generator=g)
    if content == "flat":
        lv = ((torch.arange(S, device="cuda") * 37 + seed0) % 224 + 16).to(torch.uint8)
        return lv.view(1, S, 1).expand(nslots, S, pic).contiguous()
    base = p64_amd.synth_frames_device(w, h, seed0, S, 0, 1)[0]  # [S, pic]
    out = torch.empty((nslots, S, pic), dtype=torch.uint8, device="cuda")
    s_idx = torch.arange(S, device="cuda")
    vx = torch.where(s_idx % 2 == 0, 15, -15)
    vy = torch.where((s_idx // 2) % 2 == 0, 15, -15)
    planes = ((0, w, h, 1), (w * h, w // 2, h // 2, 2), (w * h + w * h // 4, w // 2, h // 2, 2))
    for t in range(nslots):
        for off, pw, ph, div in planes:
            src = base[:, off:off + pw * ph].view(S, ph, pw)
            rows = (torch.arange(ph, device="cuda")[None, :] - (t * vy // div)[:, None]) % ph
            cols = (torch.arange(pw, device="cuda")[None, :] - (t * vx // div)[:, None]) % pw
            moved = src[s_idx[:, None, None], rows[:, :, None], cols[:, None, :]].to(torch.int16)
            noise = torch.randint(-3, 4, moved.shape, dtype=torch.int16, device="cuda", generator=g)
            out[t, :, off:off + pw * ph] = (moved + noise).clamp_(0, 255).to(torch.uint8).view(S, -1)
    return out


def _pow2_quant(q):
    """the library's packed-quantiser instances: a uniform q with 16q a power
    of two (k_block.hip qlevel_pk2)"""
    return q in (1, 2, 4, 8, 16)


def intra_kernel_name(q):
    """k_intra_mbg's instance for a uniform q (p64k::intra_mbg): <QMB, CLAMP,
    POW2> as rocprof prints it"""
    clamp = "false" if q >= 5 else "true"
    return f"k_intra_mbg<false, {clamp}, {'true' if _pow2_quant(q) else 'false'}, false>"


def inter_kernel_name(q):
    """k_inter_mbg's instance for a uniform q without overrides and without
    the entropy coder's bit counts (p64k::inter_mbg): <QMB, OVR, POW2, BITS>"""
    return "k_inter_mbg<false, false, %s, false>" % ("true" if _pow2_quant(q) else "false")


def content_key(args, base):
    """Key of a workload in the tracked profiles (PMC passes, rocprof timed
    regions, executed SAD counts): the builder's synth content has none, the
    others their name."""
    return base if args.content == "synth" else f"{base}_{args.content}"


def load_pmc(path, workload_key):
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(workload_key)
        return e if e else None
    except (OSError, ValueError):
        return None


def timing_note(args, root=False):
    if root and args.gather == "coded" and not args.eager and os.environ.get("P64_FEED_GRAPHS", "0") != "0":
        return "HIP events around each step's graph replay (encode + entropy coder)"
    if args.eager or root:
        return "HIP events around each launch (kernel + launch gap)"
    return "HIP events around the replay of a graph of the K launches, / K (includes the inter-kernel boundary)"


def roofline(bytes_per_launch, kavg, kernel, pmc=None, **extra):
    gbs = bytes_per_launch / kavg / 1e9
    r = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(gbs / HBM_PEAK_GBS, 5), "traffic": (pmc or {}).get("hbm_bytes_per_launch"),
         "kernel": kernel, "kernel_avg_us": round(kavg * 1e6, 2),
         "algorithmic_bytes_per_launch": int(bytes_per_launch)}
    r.update(extra)
    return r


# ---------------------------------------------------------------------------
# the timed configurations

def timed_region(torch, dist, world, steps, t_first, launch, pre=None, post=None, graph=True,
                 spinup_ms=0, spin=None, finish=None):
    """The K timed steps, bracketed by barrier + synchronize on both sides.

    launch(t) issues step t's kernel on torch's current stream (the library
    launches on it).  graph=True captures the K launches once into a HIP graph
    (torch.cuda.CUDAGraph) and times its replay: the kernels run back to back
    with no host launch cost between them (a step of the intra or decode
    config is shorter than a Python launch).  Eagerly (graph=False, and always
    when pre/post collectives are part of the step) each launch is bracketed by
    its own events, so collectives do not count as kernel time.

    Steady state: the chip raises its clocks over tens of ms of load and drops
    them when idle (the capture and the verification snapshot before the
    region leave it idle for ~12 ms); a 20-step region (3.6 ms) measured from
    there ran 12% slower than the same kernels after ~25 ms of load
    (profiles/r04a_clock_sweep.txt).  So, when spin is given (dict: init()
    allocates scratch outputs, reset() copies the closed-loop state into
    scratch, launch(t) issues step t exactly as launch does but into the
    scratch), [reset + the K scratch steps] is replayed back to back for >=
    spinup_ms -- every replay the same work as the timed one, outputs
    discarded -- and the timed region follows.  Nothing the timed steps read
    is produced by the spin-up, and no work is dropped from them.
    spin["split"] = (first, rest, full(t, k), part(t, k)), if given, splits
    the step's time between its two kernels: a graph of the K full steps
    (full: step t, the k-th, keeping what the second kernel needs) and one
    of the second kernels alone (part), each replayed once after a reset and
    timed with HIP events; the first kernel's time is the difference.
    A 50-us clock probe after the region reads the clock the chip was left
    at (box-to-box spread).
    finish(), if given, runs after the last step inside the region (the fed
    path's gather of its last step, CodedFeed).
    Returns (wall seconds of the timed region, mean kernel seconds per step,
    steady-state record)."""
    import p64_amd
    if pre is not None or post is not None:
        graph = False
    st = {"spinup_ms": spinup_ms if spin else 0, "spinup_replays": 0}

    def capture(fn, first=None):
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            if first is not None:
                first()
            for k in range(steps):
                fn(t_first + k)
        torch.cuda.synchronize()
        return gr

    g = capture(launch) if graph else None
    if spin is not None and spinup_ms > 0:
        spin["init"]()
        gs = capture(spin["launch"], spin["reset"]) if graph else None

        def run():
            if graph:
                gs.replay()
            else:
                spin["reset"]()
                for k in range(steps):
                    spin["launch"](t_first + k)
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        one = time.perf_counter() - t0
        n = max(0, int(spinup_ms * 1e-3 / max(one, 1e-6) + 0.999) - 1)
        for _ in range(n):  # back to back, no host synchronisation between them
            run()
        torch.cuda.synchronize()
        st["spinup_replays"] = 1 + n
        st["spinup_ms_actual"] = round((time.perf_counter() - t0) * 1e3, 1)
        if spin.get("split") and graph:  # the step's kernels apart, at steady clocks
            first, rest, full, part = spin["split"]
            times = {}
            for nm, fn in (("step", full), (rest, part)):
                gp = capture(lambda t, fn=fn: fn(t, t - t_first))
                spin["reset"]()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                gp.replay()
                b.record()
                torch.cuda.synchronize()
                times[nm] = a.elapsed_time(b) * 1e3 / steps
                del gp
            st["kernels_us_live"] = {first: round(times["step"] - times[rest], 2), rest: round(times[rest], 2)}
            st["kernels_us_live_note"] = (
                f"graphs of the K steps right after the spin-up (same steps and state as the timed "
                f"region), HIP events around each replay, / K: the whole step ({times['step']:.2f} us) "
                f"recording each step's ME records, then {rest} alone from those records "
                f"(P64GPU_FLAG_ME_GIVEN); {first} = the difference")
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(1 if graph else steps)]
    # torch creates an event's HIP event at its first record(): recorded once
    # here, so that creation (~100 us of host time the first time in a process,
    # measured as the intra line's 45.2 vs 38.0 us per step) is not inside the
    # timed region
    for a, b in ev:
        a.record()
        b.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if graph:
        ev[0][0].record()
        g.replay()
        ev[0][1].record()
    else:
        for k in range(steps):
            t = t_first + k
            if pre is not None:
                pre(t)
            ev[k][0].record()
            launch(t)
            ev[k][1].record()
            if post is not None:
                post(t)
        if finish is not None:
            finish()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st["clock_mhz_after"] = p64_amd.clock_probe(50)
    kern = sum(a.elapsed_time(b) for a, b in ev) * 1e-3 / steps
    del g
    return elapsed, kern, st


def coded_level_bytes(torch, mb):
    """128 bytes per transmitted block of the records mb [..., 4]: MTYPE with
    coefficients and (for MTYPEs with a CBP) its CBP bit set."""
    mt = mb[..., 0].reshape(-1).long()
    cbp = mb[..., 1].reshape(-1).long() & 63
    tc = torch.tensor([1, 1, 1, 1, 0, 1, 1, 0, 1, 1], device=mb.device)[mt]
    has_cbp = torch.tensor([0, 0, 1, 1, 0, 1, 1, 0, 1, 1], device=mb.device)[mt]
    cbp = torch.where(has_cbp == 1, cbp, torch.full_like(cbp, 63))
    nblk = sum(((cbp >> b) & 1) for b in range(6)) * tc
    return int(128 * nblk.sum().item())


def decode_bytes(torch, mb, nmb_all):
    """Algorithmic HBM bytes of one k_recon_mbg launch over records mb
    [nmb_all, 4] (all MBs coded): record + UseQuant + coded flag, the levels of
    coded blocks, the prediction source of non-intra MBs, the recon write."""
    inter = (mb[..., 0].reshape(-1).long() >= 2).long()
    return int(6 * nmb_all + coded_level_bytes(torch, mb) + 384 * inter.sum().item() + 384 * nmb_all)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args, argv))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}: refusing to report")
    if args.dry:
        return dry_main(args, rank, world)

    cpus = {}
    if rank == 0 and world == 1 and not args.no_cpu:
        legs = {"inter": ["inter"] + ([] if args.no_extra else ["intra", "decode"]),
                "4cif": ["inter"], "intra": ["intra"], "decode": ["decode"]}[args.config]
        cpus = cpu_baselines(args, legs)
    cpu = cpus.get(args.config if args.config in ("intra", "decode") else "inter")

    import numpy as np
    import torch
    import torch.distributed as dist

    import p64_amd

    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    ranks = rank_info(world, rank, local, dist, torch)

    w, h = args.width, args.height
    nmb = (w // 16) * (h // 16)
    pic = w * h * 3 // 2
    seed0, S = shard_seeds(rank, args.streams)
    nslots = min(1 + args.warmup + args.steps, MAX_SLOTS)
    slot = lambda t: t % nslots  # noqa: E731
    mode = p64_amd.ME_FULL if args.mode == "full" else p64_amd.ME_TSS
    sys.path.insert(0, os.path.join(REPO, "oracle"))

    root = args.feed == "root" and args.config in ("inter", "4cif")
    if root:  # rank 0 generates every rank's pictures; the others receive per step
        all_frames = (make_inputs(torch, p64_amd, args.content, w, h, 1, world * S, nslots)
                      if rank == 0 else None)
        frames = torch.empty((nslots, S, pic), dtype=torch.uint8, device="cuda")
        lv = rank == 0 and args.gather == "levels"
        coef_bufs = ([torch.empty((S, nmb, 6, 64), dtype=torch.int16, device="cuda")
                      for _ in range(world)] if lv else None)
        mb_bufs = [torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda") for _ in range(world)] if lv else None
    else:
        frames = make_inputs(torch, p64_amd, args.content, w, h, seed0, S, nslots)

    result = {}
    if args.config == "intra":
        result = run_intra(args, torch, dist, np, p64_amd, world, frames, S, nmb, pic, nslots)
    elif args.config == "decode":
        enc = encode_all(args, torch, p64_amd, frames, S, nmb, pic, nslots, mode)
        result = run_decode(args, torch, dist, np, p64_amd, world, enc, S, nmb, pic)
    else:
        keep = not args.no_extra and world == 1 and not root
        rec = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
        li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
        # levels and records of every step stay resident when the decode config
        # is measured from them afterwards (nslots x 78 MB at S=256 CIF);
        # otherwise the checked pictures (vt, last) get level buffers of their
        # own.  The level buffers start as LEVEL_SENTINEL: an inter picture
        # stores exactly the blocks its nonzero-block mask names
        # (include/p64gpu.h), so every other block must still hold it.
        vt, last = args.warmup, args.warmup + args.steps
        # --feed root --gather coded: the unchecked steps alternate between two
        # output sets (0 and 3), so step t's coder (on the feed's side stream)
        # reads a set step t+1's encode does not write
        alt = root and args.gather == "coded"
        ncoef = nslots if keep else (4 if alt else 3)
        coef_all = torch.full((ncoef, S, nmb, 6, 64), LEVEL_SENTINEL, dtype=torch.int16, device="cuda")
        nz_all = torch.empty((ncoef, S, nmb), dtype=torch.uint8, device="cuda")
        mb_all = torch.empty((ncoef, S, nmb, 4), dtype=torch.int8, device="cuda")
        me = torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda")
        # --feed root --gather coded: the encoder counts the coded bits for the in-step VLC
        vb_root = None  # (--feed root codes with the coder's own counts: with_vlc measures it faster)

        def out_of(t):
            i = slot(t) if keep else (1 if t == vt else (2 if t == last else (3 * (t % 2) if alt else 0)))
            return p64_amd.FrameBatchOut(coef=coef_all[i], mb=mb_all[i], me=me, nz=nz_all[i], vlc_bits=vb_root)
        # the checked pictures' buffers were written by no earlier step
        fresh = {t: (not keep) or (1 + args.warmup + args.steps <= nslots) for t in (vt, last)}

        def pre(t):  # --feed root: this step's pictures from rank 0
            scatter_pictures(world, rank, all_frames[slot(t)] if rank == 0 else None, frames[slot(t)])

        def launch(t, vlc_bits=None):  # vlc_bits: the entropy coder's block bits, counted by the encoder
            o = out_of(t)
            if vlc_bits is not None:
                o = dataclasses.replace(o, vlc_bits=vlc_bits)
            p64_amd.encode_frames(frames[slot(t)].reshape(-1), rec[(t + 1) % 2], rec[t % 2], li,
                                  width=w, height=h, intra=(t == 0), quant=args.quant,
                                  me_mode=mode, search_limit=args.search_limit, out=o)

        feed = None
        if root and args.gather == "coded":  # each rank entropy-codes its pictures in the step
            from p64_amd import stream as p64s
            keep_seqs = ([i for i in VERIFY_SEQS if i < S] + [r * S for r in range(1, world)]
                         if rank == 0 and not args.no_verify else [])
            feed = CodedFeed(torch, p64s, world, rank, S, w, h, args.quant, keep=keep_seqs)

        def post(t):  # --feed root: the coded pictures (or levels and records) back to rank 0
            o = out_of(t)
            if args.gather == "levels":
                gather_outputs(world, rank, o.coef, coef_bufs)
                gather_outputs(world, rank, o.mb, mb_bufs)
                return
            feed.code(t, o)  # (gathers the previous step's pictures)

        def step(t, vlc_bits=None):
            if root:
                pre(t)
            if feed is not None:
                feed.before_encode(t)
            launch(t, vlc_bits)
            if root:
                post(t)

        # steady-state spin-up (timed_region): the same launches into scratch
        kme, kin = "k_motion<%d>" % (2 if args.mode == "full" else 1), inter_kernel_name(args.quant)
        sp = {}

        def spin_init():
            sp["rec"] = [torch.empty_like(r) for r in rec]
            sp["li"] = torch.empty_like(li)
            sp["out"] = p64_amd.FrameBatchOut(coef=torch.empty_like(coef_all[0]),
                                              mb=torch.empty_like(mb_all[0]), me=torch.empty_like(me),
                                              nz=torch.empty_like(nz_all[0]))

        def spin_reset():
            for a, b in zip(sp["rec"], rec):
                a.copy_(b)
            sp["li"].copy_(li)

        def spin_launch(t):
            p64_amd.encode_frames(frames[slot(t)].reshape(-1), sp["rec"][(t + 1) % 2], sp["rec"][t % 2],
                                  sp["li"], width=w, height=h, intra=False, quant=args.quant,
                                  me_mode=mode, search_limit=args.search_limit, out=sp["out"])

        def spin_out(k):  # scratch outputs with step k's own ME records
            if "mes" not in sp:
                sp["mes"] = [torch.empty_like(me) for _ in range(args.steps)]
            return p64_amd.FrameBatchOut(coef=sp["out"].coef, mb=sp["out"].mb, me=sp["mes"][k],
                                         nz=sp["out"].nz)

        def spin_full(t, k):  # the whole step, its ME records kept
            p64_amd.encode_frames(frames[slot(t)].reshape(-1), sp["rec"][(t + 1) % 2], sp["rec"][t % 2],
                                  sp["li"], width=w, height=h, intra=False, quant=args.quant,
                                  me_mode=mode, search_limit=args.search_limit, out=spin_out(k))

        def spin_rest(t, k):  # the step after the search, from those records
            p64_amd.encode_frames(frames[slot(t)].reshape(-1), sp["rec"][(t + 1) % 2], sp["rec"][t % 2],
                                  sp["li"], width=w, height=h, intra=False, quant=args.quant,
                                  me_mode=mode, search_limit=args.search_limit, out=spin_out(k),
                                  me_given=True)

        for t in range(1 + args.warmup):  # intra picture + warmup, untimed
            step(t)
        timed_launch, timed_post = launch, (post if root else None)
        feed_graphs = feed is not None and not args.eager and os.environ.get("P64_FEED_GRAPHS", "0") != "0"
        if feed is not None and not feed_graphs:
            # eager fed steps with every launch's arguments checked and packed
            # before the region (p64_amd.prepare_encode / stream.prepare_vlc):
            # the host issues the step without the wrappers' per-call checks
            prep = {}
            for t in range(1 + args.warmup, 1 + args.warmup + args.steps):
                o = out_of(t)
                enc = p64_amd.prepare_encode(frames[slot(t)].reshape(-1), rec[(t + 1) % 2], rec[t % 2], li,
                                             width=w, height=h, intra=False, quant=args.quant, me_mode=mode,
                                             search_limit=args.search_limit, out=o)
                vlc, vbits = p64s.prepare_vlc(o.mb, o.coef, feed.gq, feed.trs[t % 32], width=w, height=h,
                                              buffers=feed.bufs[t % 2], blk_bits=o.vlc_bits,
                                              seq_bits=feed.seq_bits, max_bits=feed.mx[t % 2],
                                              stream=feed.side if feed.fork else None)
                prep[t] = (enc, vlc, vbits)

            def timed_launch(t):
                feed.before_encode(t)
                prep[t][0]()

            def timed_post(t):
                feed.code(t, None, vlc=(prep[t][1], prep[t][2]))
        if feed_graphs:
            feed.fork = False  # (the coder inside each step's graph, on the encode stream)
            # --feed root, coded: each timed step's device work (encode + coder
            # + the phase bookkeeping) captured as its own HIP graph before the
            # region and replayed in the step, so the host issues four calls a
            # step (scatter, replay, event, the previous step's gather) instead
            # of ~15 launches; nothing is skipped: every graph runs once, in
            # order, inside the timed region (the scatter and gather stay eager:
            # they are the collectives)
            step_graphs = {}
            for t in range(1 + args.warmup, 1 + args.warmup + args.steps):
                torch.cuda.synchronize()
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr):
                    launch(t)
                    feed.code_gpu(t, out_of(t))
                step_graphs[t] = gr
            # each graph replays once: uploaded now (hipGraphUpload), so its
            # first launch inside the region does not pay for the upload
            # (measured 640 against ~240 us per step without it)
            hip_rt = None
            with open("/proc/self/maps") as f:
                for ln in f:
                    if "libamdhip64" in ln:
                        import ctypes
                        hip_rt = ctypes.CDLL(ln.split()[-1])
                        break
            for gr in step_graphs.values():
                ex = gr.raw_cuda_graph_exec()
                if hip_rt is not None and ex:
                    hip_rt.hipGraphUpload(ctypes.c_void_p(ex),
                                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            torch.cuda.synchronize()

            dbg = os.environ.get("P64_FEED_SYNC", "0") != "0"  # (diagnostic: localise a fault)

            def timed_launch(t):
                torch.cuda.current_stream().wait_stream(feed.side)
                step_graphs[t].replay()
                if dbg:
                    torch.cuda.synchronize()
                    print(f"feed step {t}: replay ok", file=sys.stderr, flush=True)
                feed.code_host(t)
                if dbg:
                    torch.cuda.synchronize()
                    print(f"feed step {t}: gather ok", file=sys.stderr, flush=True)
            timed_post = None
        if feed is not None:
            # the scatters of steps t+1 and t+2 are issued during step t on the
            # feed's side stream (at most 3 slots live, all distinct), so a step's
            # pictures were queued two steps ahead -- behind the coder of step
            # t-1, which shares the GPU with step t's encode and finishes late
            # (one step ahead, the encode of t+1 waited for that coder and the
            # scatter behind it: 68 us idle per step, profiles/r06m_fed_trace.txt);
            # the first timed step scatters in place, so the region holds
            # exactly K scatters.  (Not a stream of its own: a fourth stream
            # shares a hardware queue with the encode stream -- GPU_MAX_HW_QUEUES
            # = 4 -- and serialised the gathers behind the encodes: 579 against
            # 298 us per step.)  Three events, created once, rotate.
            assert nslots >= 3
            pf_ev = [torch.cuda.Event() for _ in range(3)]
            pf_done = set()
            t_last = args.warmup + args.steps
            ahead = int(os.environ.get("P64_FEED_AHEAD", "2"))  # (1: round 6's first form)

            def timed_pre(t):
                if t not in pf_done:
                    pre(t)
                else:
                    torch.cuda.current_stream().wait_event(pf_ev[t % 3])
                    pf_done.discard(t)
                for u in range(t + 1, min(t + ahead, t_last) + 1):
                    if u not in pf_done:
                        with torch.cuda.stream(feed.side):
                            pre(u)
                            pf_ev[u % 3].record(feed.side)
                        pf_done.add(u)
        feed_host = None
        if feed is not None:  # host seconds spent issuing each part of the fed step (incl. its waits)
            feed_host = {"pre": 0.0, "launch": 0.0, "post": 0.0}

            def host_timed(fn, key):
                if fn is None:
                    return None

                def f(t):
                    a = time.perf_counter()
                    fn(t)
                    feed_host[key] += time.perf_counter() - a
                return f
            timed_pre = host_timed(timed_pre, "pre")
            timed_launch = host_timed(timed_launch, "launch")
            timed_post = host_timed(timed_post, "post")
        # the checked sequences (VERIFY_SEQS: one of each synth seed class) after
        # the warmup, checked against the oracle after the timed region
        seqs = [i for i in VERIFY_SEQS if i < S]
        snap = {}
        if rank == 0 and not args.no_verify:
            snap[vt] = snapshot(out_of(vt), me, rec[vt % 2], seqs, pic)
        t_first = 1 + args.warmup
        elapsed, kavg, clk = timed_region(torch, dist, world, args.steps, t_first, timed_launch,
                                          (timed_pre if feed is not None else pre)
                                          if root else None, timed_post,
                                          graph=not args.eager, spinup_ms=args.spinup_ms,
                                          spin={"init": spin_init, "reset": spin_reset,
                                                "launch": spin_launch,
                                                "split": (kme, kin, spin_full, spin_rest)},
                                          finish=feed.finish if feed is not None else None)
        sp.clear()
        tmax = max_over_ranks(elapsed, world, device="cuda")
        assert last == t_first + args.steps - 1
        lvl_bytes = coded_level_bytes(torch, out_of(last).mb)  # (the last step's records)

        verified, ok = None, True
        if rank == 0 and not args.no_verify:
            # closed loop: every picture feeds the next, so matching one picture's
            # outputs and reconstruction pins the whole chain before it
            if nmb * (last + 1) <= VERIFY_MAX_MBS:
                snap[last] = snapshot(out_of(last), me, rec[last % 2], seqs, pic)
            src = all_frames if root else frames
            verified = verify_sequences(args, p64_amd, src, slot, seqs, snap, fresh, w, h, mode)
            ok = verified["ok"]
            if feed is not None and feed.keep:  # the gathered coded pictures, stitched per sequence
                coded = verify_coded(args, p64_amd, p64s, src, slot,
                                     feed.streams(p64s.format_of(w, h), (last + 1) % 32), last, w, h, mode)
                verified["coded_verified"] = coded["ok"]
                verified["coded"] = coded
                ok = ok and coded["ok"]
        if not all_ranks_ok(ok, world, device="cuda"):
            raise SystemExit("bench: GPU output differs from the oracle -- refusing to report")

        extra = None
        if keep:  # the other two configs on the same pictures and levels (before the
            # entropy-coding re-run below rewrites some of those levels)
            enc = {"coef": coef_all, "mb": mb_all, "recon_last": rec[last % 2], "last": last}
            extra = {
                "intra": strip(run_intra(args, torch, dist, np, p64_amd, world, frames, S, nmb, pic,
                                         nslots)),
                "decode": strip(run_decode(args, torch, dist, np, p64_amd, world, enc, S, nmb, pic)),
            }
            for leg in ("intra", "decode"):
                extra[leg]["cpu_baseline"] = cpus.get(leg)

        with_vlc = None
        if not args.no_vlc:
            def enc_vlc(t, o, **kw):
                p64_amd.encode_frames(frames[slot(t)].reshape(-1), rec[(t + 1) % 2], rec[t % 2], li,
                                      width=w, height=h, intra=False, quant=args.quant, me_mode=mode,
                                      search_limit=args.search_limit, out=o, **kw)
            with_vlc = measure_vlc(args, torch, p64_amd, enc_vlc, S, nmb, w, h)
        other = None
        if keep and args.content == "survey" and args.config == "inter":
            other = measure_content(args, torch, dist, world, p64_amd, "synth", S, seed0, nslots, mode)

        mbs_launch = S * nmb
        value = aggregate_rate(world, mbs_launch, args.steps, tmax)
        cand = 33
        if args.mode == "full":
            hl = args.search_limit // 2
            cand = (2 * hl) * (2 * hl)
        sad_rate = mbs_launch * cand * 256 / kavg
        me_name = "FULL FastBME SL=%d" % args.search_limit if args.mode == "full" else "TSS StepBME"
        workload = (f"{w}x{h} inter, {me_name}, q={args.quant}, content {args.content}, "
                    f"closed loop, {S} sequences/GPU")
        key = content_key(args, f"{w}x{h}_{args.mode}{args.search_limit}_q{args.quant}_S{S}")
        pmc = load_pmc(args.pmc_json, key)
        pmc_me, pmc_in = load_pmc(args.pmc_json, key + "_me"), load_pmc(args.pmc_json, key + "_inter")
        if os.environ.get("P64GPU_FUSED", "0") in ("", "0"):  # split: k_motion, k_inter_mbg
            kernel = f"{kme} + {kin} (one step)"
            prof = (load_json(os.path.join(REPO, PROFILE_TIMED)) or {}).get(key) or {}
            split = {"dominant": kme,
                     "dominant_note": "k_motion is VALU-bound (roofline_sad_executed, valu_busy); the "
                                      "HBM roofline is taken over the whole step, both kernels",
                     "kernels_us_live": clk.get("kernels_us_live"),
                     "kernels_us_rocprof": ({k: prof[k] for k in (kme, kin)}
                                            if all(k in prof for k in (kme, kin)) else None),
                     "kernels_us_rocprof_source": f"{PROFILE_TIMED} (rocprofv3 --kernel-trace of "
                                                  "`bench.py --steps 20 --warmup 5 --no-cpu`, timed "
                                                  "region only: tools/timed_region.py)"}
            pmc = None  # (an entry under `key` would be the fused kernel's)
            if pmc_me and pmc_in:
                pmc = {"hbm_bytes_per_launch": pmc_me["hbm_bytes_per_launch"] +
                       pmc_in["hbm_bytes_per_launch"],
                       "valu_busy": {kme: pmc_me.get("valu_busy"), kin: pmc_in.get("valu_busy")}}
        else:
            kernel = "k_encode<%d>" % (2 if args.mode == "full" else 1)
            split = {}
        result = {
            "metric": METRICS[args.config], "value": round(value, 1),
            "ms_per_step": round(tmax / args.steps * 1e3, 4),
            "config": {"workload": workload, "content": args.content, "feed": args.feed,
                       **({"gather": args.gather} if root else {}),
                       "width": w, "height": h, "me": args.mode,
                       "search_limit": args.search_limit, "quant": args.quant,
                       "sequences_per_gpu": S, "macroblocks_per_step_per_gpu": mbs_launch,
                       "distinct_input_pictures": nslots,
                       "parallelism": (f"dp{world} (independent sequences per GPU, no data-path "
                                       f"collective)" if not root else
                                       f"dp{world} (rank 0 RCCL-scatters pictures, gathers "
                                       + ("the entropy-coded pictures (GPU VLC on each rank in the step)"
                                          if args.gather == "coded" else "levels + records")
                                       + ("; roofline times each step's device work: encode + coder, one "
                                          "graph replay per step" if feed_graphs
                                          else "; roofline times the encode launch alone") + ")")},
            "roofline": roofline(mbs_launch * BYTES_PER_MB_FIXED + lvl_bytes, kavg, kernel, pmc,
                                 algorithmic_bytes_per_mb=round(BYTES_PER_MB_FIXED + lvl_bytes / mbs_launch, 1),
                                 timing=timing_note(args, root),
                                 **split),
            "roofline_hbm_read": {
                "bound": "hbm", "achieved": round(mbs_launch * READ_BYTES_PER_MB / kavg / 1e9, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(mbs_launch * READ_BYTES_PER_MB / kavg / 1e9 / HBM_PEAK_GBS, 5),
                "algorithmic_read_bytes_per_mb": READ_BYTES_PER_MB,
                "note": "the north_star's HBM-read roofline: the bytes a step must read (current "
                        "picture 384 + previous reconstruction 384 + LastIntra 1 per MB) over the "
                        "step time"},
            "roofline_sad_exhaustive_equivalent": {
                "bound": "valu", "achieved": round(sad_rate / 1e12, 3),
                "peak": round(SAD_PEAK / 1e12, 3), "unit": "T byte-absdiff/s",
                "frac": round(sad_rate / SAD_PEAK, 4), "candidates_per_mb": cand,
                "note": "NOT a utilisation: the exhaustive search's candidates x 256 byte-absdiffs "
                        "per MB over the whole step time; the FULL kernel executes far fewer "
                        "(exact pruning, DESIGN.md 5): see roofline_sad_executed"},
            "roofline_sad_executed": sad_executed(args, key, kme, clk, mbs_launch),
            "valu_busy": (pmc or {}).get("valu_busy"),
            "valu_busy_note": VALU_BUSY_NOTE,
            "steady_state": clk,
            "with_vlc": with_vlc,
            **({"other_content": other} if other else {}),
            "verified_vs_oracle": verified,
        }
        if feed_host is not None:
            result["feed_host_us_per_step"] = {k: round(v / args.steps * 1e6, 1) for k, v in feed_host.items()}
            result["feed_host_note"] = ("host time per timed step in each part of the fed step (Python wrappers, "
                                        "launches, event waits and, at N>1, the gather's size read-back)")
        if extra:
            result["configs"] = extra

    if world > 1:
        dist.destroy_process_group()
    if rank != 0:
        return
    line = {
        "metric": result.pop("metric"),
        "value": result.pop("value"),
        "unit": "macroblocks/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": result.pop("ms_per_step"),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": (f"synthetic ({args.content}: seeded, generated on device"
                 + ("; SURVEY.md 8(d)'s texture, motion and noise" if args.content == "survey" else "") + ")"),
    }
    line.update(result)
    line["ranks"] = ranks
    if cpu is not None and line.get("with_vlc") and "macroblocks_per_s" in line["with_vlc"]:
        cpu["comparable_gpu_value"] = line["with_vlc"]["macroblocks_per_s"]
        cpu["comparable_note"] = ("the CPU leg includes entropy coding; with_vlc is the GPU rate "
                                  "with entropy coding (value stops at the levels)")
    line["cpu_baseline"] = cpu
    import p64_amd as _p
    if hasattr(_p.lib(), "p64gpu_vlc_check_errors_"):  # (a bounds-checked coder build, P64GPU_LIB)
        import ctypes
        e = ctypes.c_uint32(0)
        _p.lib().p64gpu_vlc_check_errors_(ctypes.byref(e))
        line["vlc_check_errors"] = int(e.value)
    print(json.dumps(line), flush=True)


LEVEL_SENTINEL = 0x5A5A  # never a level: H.261 levels are |l| <= 127 (DC 1..254)
# the sequences bench.py checks against the oracle: seeds 1, 5, 6, 7 -- with
# --content synth one of each generator class (plain, scene cut at picture 12,
# noise-free, low contrast: the dense-search class, synth_impl.h)
VERIFY_SEQS = (0, 4, 5, 6)
VERIFY_MAX_MBS = 120_000  # per sequence: the last picture is checked up to this run length


def snapshot(o, me, recon, seqs, pic):
    """Host copies of the checked sequences' outputs of one picture."""
    return {s: (o.coef[s].cpu().numpy(), o.nz[s].cpu().numpy(), o.mb[s].cpu().numpy(),
                me[s].cpu().numpy(), recon[s * pic:(s + 1) * pic].cpu().numpy()) for s in seqs}


def verify_sequences(args, p64_amd, src, slot, seqs, snap, fresh, w, h, mode):
    """The checked sequences against the CPU oracle (closed loop from picture
    0), one host thread per sequence (the oracle's C code runs without the
    GIL).  Per checked picture: MB records, ME records and reconstruction
    equal; the levels rebuilt through the nonzero-block mask (a set bit: the
    stored block, else 64 zeros) equal the oracle's whole inputbuf array
    (p64.c:823-913); the mask names exactly the oracle's blocks with a nonzero
    level; and blocks outside the mask still hold LEVEL_SENTINEL (the buffer
    was written by no other step), so nothing else was stored."""
    import oracle
    from concurrent.futures import ThreadPoolExecutor
    nmb = (w // 16) * (h // 16)
    upto = max(snap)
    oracle.lib()  # loaded (and its tables built) before the threads start

    def one(s):
        fr = [src[slot(t), s].cpu().numpy() for t in range(upto + 1)]
        outs = oracle.encode_sequence(fr, w, h, quant=args.quant, me_mode=mode,
                                      search_limit=args.search_limit)
        res = {}
        for t, per in snap.items():
            gc, gnz, gm, ge, gr = per[s]
            coef, mb, mev, recon = outs[t]
            bits = (gnz[:, None] >> (5 - np.arange(6))[None, :]) & 1  # [nmb, 6]
            want_nz = coef.reshape(nmb, 6, 64).any(axis=2)
            rebuilt = np.where(bits[:, :, None] == 1, gc, 0)
            checks = {"levels_via_mask": bool(np.array_equal(rebuilt, coef)),
                      "mask": bool(np.array_equal(bits == 1, want_nz)),
                      "mb": bool(np.array_equal(gm.view(p64_amd.MB_DTYPE).reshape(nmb), mb)),
                      "me": mev is None or bool(np.array_equal(ge.view(p64_amd.ME_DTYPE).reshape(nmb), mev)),
                      "recon": bool(np.array_equal(gr, recon))}
            if fresh.get(t):
                checks["untouched_blocks_sentinel"] = bool((gc[bits == 0] == LEVEL_SENTINEL).all())
            res[t] = checks
        return s, res

    with ThreadPoolExecutor(len(seqs)) as ex:
        got = dict(ex.map(one, seqs))
    ok = all(all(c.values()) for r in got.values() for c in r.values())
    return {"ok": ok, "pictures_checked": sorted(snap), "sequences_checked": [1 + s for s in seqs],
            "failed": {f"seed{1 + s}_t{t}": [k for k, v in c.items() if not v]
                       for s, r in got.items() for t, c in r.items() if not all(c.values())},
            "note": "per sequence (seed) vs the CPU oracle, closed loop from picture 0: records, "
                    "reconstruction, the whole level array rebuilt through the nonzero-block mask, "
                    "the mask itself, and the sentinel in every block the mask leaves out"}


def load_json(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def sad_executed(args, key, kme, clk, mbs):
    """k_motion's executed v_sad_u8 work against the instruction's peak: the
    byte-absolute-differences one launch executes on this workload (counted
    side build, profiles/sad_executed.json) over k_motion's own launch time
    (live: kernels_us_live, each kernel timed alone right after the spin-up;
    else the committed rocprof timed-region mean)."""
    cnt = (load_json(os.path.join(REPO, PROFILE_SAD)) or {}).get(key)
    us = (clk.get("kernels_us_live") or {}).get(kme)
    src = "live"
    if us is None:
        us = ((load_json(os.path.join(REPO, PROFILE_TIMED)) or {}).get(key) or {}).get(kme)
        src = PROFILE_TIMED
    if not cnt or not us or args.mode != "full":
        return None
    per_launch = cnt["byte_absdiff_per_mb"] * mbs
    rate = per_launch / (us * 1e-6)
    return {"bound": "valu", "kernel": kme, "achieved": round(rate / 1e12, 3),
            "peak": round(SAD_PEAK / 1e12, 3), "unit": "T byte-absdiff/s", "frac": round(rate / SAD_PEAK, 4),
            "executed_byte_absdiff_per_mb": round(cnt["byte_absdiff_per_mb"], 1),
            "kernel_us": us, "kernel_us_source": src,
            "note": "executed v_sad_u8 lane-instructions x 4 (counted by tools/sad_count.py on this "
                    "workload, profiles/sad_executed.json) over k_motion's launch time; the rest of "
                    "k_motion's issue is the bound map, addressing and reductions (valu_busy). The "
                    "fraction falls when the pruning improves (fewer SADs for the same answer): on "
                    "survey content the bound leaves fewer full SADs than on synth, so 0.16 here "
                    "against 0.29 there at similar kernel times. k_motion's utilisation is valu_busy "
                    "(VALU issue, PMC-derived; DESIGN.md 9a item 3 shows +64 VALU per MB costing "
                    "80-90% of their issue time)"}


def strip(r):
    """A nested config line: everything but the top-level contract keys."""
    return {k: v for k, v in r.items() if k not in ("with_vlc",)}


def measure_vlc(args, torch, p64_amd, enc, S, nmb, w, h):
    """The encode steps followed by entropy coding on the device (p64vlc.hip):
    the whole-encoder rate to .p64 bits, measured after the metric (it re-runs
    steps, so the closed-loop state is not reused).  enc(t, o) encodes step
    t's pictures into the FrameBatchOut o (the caller's closed loop).  Per
    step: the encode launches on the main stream, then the entropy coder's
    launch (counting the blocks' bits itself, or taking the encoder's counts:
    both measured), storing every picture's bit count straight into pinned
    host memory, FORKED onto a side stream, so step t's coder runs concurrently
    with step t+1's encode (round 6: the coder reads only step t's records
    and levels; two output sets alternate, and an encode waits for the coder
    that read its set two steps before); the side stream joins at the end.
    The steps are captured in one HIP graph (as the metric's steps are),
    replayed for the spin-up, then once more wall-clock timed.  Afterwards one
    more step runs eagerly and its coded pictures are compared byte for byte
    with the host writer over the same records (sequences 0 and S-1): a
    mismatch ends the bench (SystemExit, no line)."""
    try:
        from p64_amd import stream as p64s
        ngob = nmb // 33
        gq = torch.full((S, ngob), args.quant, dtype=torch.uint8, device="cuda")
        bufs = p64s.vlc_buffers(S, w, h)
        vsteps = min(args.steps, 8)
        outs = [p64_amd.FrameBatchOut(coef=torch.zeros((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                                      mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                                      me=torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda"),
                                      nz=torch.empty((S, nmb), dtype=torch.uint8, device="cuda"),
                                      vlc_bits=torch.empty((S, nmb, 8), dtype=torch.int16, device="cuda"))
                for _ in range(2)]
        trs = [torch.full((S,), (1 + args.warmup + k) % 32, dtype=torch.int32, device="cuda")
               for k in range(vsteps)]
        host = torch.empty((vsteps, S), dtype=torch.int32, pin_memory=True)
        p64s.vlc_pictures(outs[0].mb, outs[0].coef, gq, trs[0], width=w, height=h, buffers=bufs,
                          host_bits=False)  # first call: table upload (records not yet written)
        torch.cuda.synchronize()
        vlc_ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        side = torch.cuda.Stream()

        def coder(k, o, given):
            # each picture's bit count stored by the coder straight into the
            # pinned host row (device-addressable: p64gpu_vlc_args, ABI v3) --
            # no copy launch after it
            p64s.vlc_pictures(o.mb, o.coef, gq, trs[k], width=w, height=h, buffers=(bufs[0], host[k], bufs[2]),
                              host_bits=False, blk_bits=o.vlc_bits if given else None)

        def run(given, split):
            def out(k):
                o = outs[k % 2]
                return o if given else dataclasses.replace(o, vlc_bits=None)
            ev_enc = [torch.cuda.Event() for _ in range(vsteps)]
            ev_done = [torch.cuda.Event() for _ in range(vsteps)]
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                main = torch.cuda.current_stream()
                for k in range(vsteps):
                    if not split:
                        if k >= 2:
                            main.wait_event(ev_done[k - 2])  # (that coder has read this output set)
                        enc(1 + args.warmup + k, out(k))
                        ev_enc[k].record(main)
                        side.wait_event(ev_enc[k])
                        with torch.cuda.stream(side):
                            coder(k, outs[k % 2], given)
                            ev_done[k].record(side)
                        continue
                    # split: step k's search (P64GPU_FLAG_SEARCH_ONLY, writes only
                    # the ME records), then step k-1's coder on the side stream
                    # beside step k's second half (ME_GIVEN), which is HBM- and
                    # latency-bound where the search is VALU-bound
                    enc(1 + args.warmup + k, out(k), search_only=True)
                    ev_enc[k].record(main)
                    if k >= 1:
                        side.wait_event(ev_enc[k])
                        with torch.cuda.stream(side):
                            coder(k - 1, outs[(k - 1) % 2], given)
                            ev_done[k - 1].record(side)
                    if k >= 2:
                        main.wait_event(ev_done[k - 2])  # (that coder has read this output set)
                    enc(1 + args.warmup + k, out(k), me_given=True)
                if split:
                    side.wait_stream(main)
                    with torch.cuda.stream(side):
                        coder(vsteps - 1, outs[(vsteps - 1) % 2], given)
                main.wait_stream(side)
            torch.cuda.synchronize()
            # the first replay uploads the graph; then replays for >= spinup_ms
            # (the chip ramps its clocks over tens of ms, timed_region), the
            # last one timed (each replay continues the closed loop: its first
            # step predicts from the previous replay's last picture)
            t0 = time.perf_counter()
            while True:
                g.replay()
                torch.cuda.synchronize()
                if (time.perf_counter() - t0) * 1e3 >= args.spinup_ms:
                    break
            t1 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t1
            del g
            hb = host.numpy().astype(np.int64) & 0xFFFFFFFF
            if (hb == 0xFFFFFFFF).any():
                raise RuntimeError("vlc: invalid record or overflow")
            # one more step eagerly: the coder's launch timed alone, and its
            # pictures against the host writer
            k = vsteps - 1
            o = out(k)
            enc(1 + args.warmup + k, o)
            vlc_ev[0].record()
            coder(k, outs[k % 2], given)
            vlc_ev[1].record()
            torch.cuda.synchronize()
            check_coded(p64s, outs[k % 2], bufs, host[k].numpy(), trs[k], args.quant, w, h, (0, S - 1))
            return {"macroblocks_per_s": round(S * nmb * vsteps / dt, 1),
                    "ms_per_step": round(dt / vsteps * 1e3, 4),
                    "vlc_ms_last_step": round(vlc_ev[0].elapsed_time(vlc_ev[1]), 4),
                    "avg_bits_per_mb": round(float(hb.sum()) / (S * nmb * vsteps), 2)}

        # the ways to the bits: the encoder counts every transmitted block's
        # bits (vlc_bits) and the coder takes them, or the coder counts; the
        # coder beside the next step's whole encode, or beside its second half
        paths = {}
        for name, given, split in (("encoder counts", True, False), ("the coder counts", False, False),
                                   ("encoder counts, coder beside the second half", True, True),
                                   ("the coder counts, coder beside the second half", False, True)):
            paths[name] = run(given, split)
        name = min(paths, key=lambda n: paths[n]["ms_per_step"])
        res = dict(paths[name])
        res["path"] = name
        res["other_paths"] = {n: {"macroblocks_per_s": v["macroblocks_per_s"], "ms_per_step": v["ms_per_step"]}
                              for n, v in paths.items() if n != name}
        res["coded_checked"] = {"sequences": [1, S], "vs": "host writer (p64s_write_picture) over the same records",
                                "ok": True}
        res["note"] = ("encode launches + GPU entropy coding (one launch after the status words' zeroing "
                       "kernel: each workgroup of 40 MBs counts or takes its bits, finds its start by a "
                       "decoupled look-back, writes its words) per step, the coder -- its bit counts "
                       "stored straight into pinned host memory -- forked onto a side stream (concurrent "
                       "with the next step's encode, or with its second half when split: "
                       "P64GPU_FLAG_SEARCH_ONLY + ME_GIVEN), the steps "
                       "replayed as one HIP graph after a spin-up; the fastest of four paths (path / "
                       "other_paths); not part of `value`")
        return res
    except Exception as e:  # never let the extra measurement cost the bench line
        return {"error": str(e)[:200]}


def check_coded(p64s, o, bufs, bits, tr, quant, w, h, seqs):
    """The coder's pictures of sequences `seqs` (bytes in bufs[0], counts in
    bits) equal the host writer's over the same records, bit for bit (ADVICE
    r05: a timing-dependent coder fault must not pass unnoticed); SystemExit
    otherwise."""
    fmt = p64s.format_of(w, h)
    data = bufs[0].cpu().numpy()
    mb, coef, trh = o.mb.cpu().numpy(), o.coef.cpu().numpy(), tr.cpu().numpy()
    for s in seqs:
        wr = p64s.Writer(fmt)
        wr.write_picture(int(trh[s]), mb[s], coef[s], quant)
        nb, b = wr.bits(), int(bits[s]) & 0xFFFFFFFF
        full = wr.data()
        nbytes = (b + 7) // 8
        gpu = int.from_bytes(data[s, :nbytes].tobytes(), "big") >> (nbytes * 8 - b) if b else 0
        if b != nb or gpu >> (nb - 8 * len(full)) != int.from_bytes(full, "big"):
            raise SystemExit(f"bench: GPU entropy coder differs from the host writer (sequence {s + 1}) "
                             f"-- refusing to report")


def measure_content(args, torch, dist, world, p64_amd, content, S, seed0, nslots, mode):
    """The same inter steps on another content (the secondary line: round 4's
    headline content `synth`), timed the same way, for comparison across
    rounds; not part of `value`."""
    try:
        w, h = args.width, args.height
        nmb, pic = (w // 16) * (h // 16), w * h * 3 // 2
        frames = make_inputs(torch, p64_amd, content, w, h, seed0, S, nslots)
        rec = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
        li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")

        def outs():
            return p64_amd.FrameBatchOut(coef=torch.empty((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                                         mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"),
                                         me=torch.empty((S, nmb, 7), dtype=torch.int32, device="cuda"),
                                         nz=torch.empty((S, nmb), dtype=torch.uint8, device="cuda"))
        out = outs()

        def launch(t, r=rec, l=li, o=out, **kw):
            p64_amd.encode_frames(frames[t % nslots].reshape(-1), r[(t + 1) % 2], r[t % 2], l, width=w,
                                  height=h, intra=(t == 0), quant=args.quant, me_mode=mode,
                                  search_limit=args.search_limit, out=o, **kw)
        for t in range(1 + args.warmup):
            launch(t)
        sp = {}

        def spin_init():
            sp["rec"], sp["li"], sp["out"] = [torch.empty_like(r) for r in rec], torch.empty_like(li), outs()

        def spin_reset():
            for a, b in zip(sp["rec"], rec):
                a.copy_(b)
            sp["li"].copy_(li)

        elapsed, _, clk = timed_region(torch, dist, world, args.steps, 1 + args.warmup, launch,
                                       graph=not args.eager, spinup_ms=args.spinup_ms,
                                       spin={"init": spin_init, "reset": spin_reset,
                                             "launch": lambda t: launch(t, sp["rec"], sp["li"], sp["out"])})
        tmax = max_over_ranks(elapsed, world, device="cuda")
        sp.clear()
        res = {"content": content, "value": round(aggregate_rate(world, S * nmb, args.steps, tmax), 1),
               "ms_per_step": round(tmax / args.steps * 1e3, 4),
               "clock_mhz_after": clk.get("clock_mhz_after"),
               "note": "the same inter steps (closed loop, K steps in one graph) on this content; "
                       "round 4's headline content was synth"}
        if not args.no_vlc:  # and the whole encoder to bits on it (round 4's with_vlc was on synth)
            res["with_vlc"] = measure_vlc(args, torch, p64_amd, lambda t, o, **kw: launch(t, o=o, **kw), S, nmb,
                                          w, h)
        return res
    except Exception as e:  # never let the extra measurement cost the bench line
        return {"content": content, "error": str(e)[:200]}


def run_intra(args, torch, dist, np, p64_amd, world, frames, S, nmb, pic, nslots):
    """configs[1]: every step intra-codes a distinct picture of every sequence."""
    w, h = args.width, args.height
    rec = torch.empty(S * pic, dtype=torch.uint8, device="cuda")
    li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
    out = p64_amd.FrameBatchOut(coef=torch.empty((S, nmb, 6, 64), dtype=torch.int16, device="cuda"),
                                mb=torch.empty((S, nmb, 4), dtype=torch.int8, device="cuda"), me=None)
    def step(t):
        p64_amd.encode_frames(frames[t % nslots].reshape(-1), None, rec, li, width=w, height=h,
                              intra=True, quant=args.quant, out=out)

    sp = {}

    def spin_init():
        sp["rec"], sp["li"] = torch.empty_like(rec), torch.empty_like(li)
        sp["out"] = p64_amd.FrameBatchOut(coef=torch.empty_like(out.coef), mb=torch.empty_like(out.mb), me=None)

    def spin_reset():
        sp["li"].copy_(li)

    def spin_step(t):
        p64_amd.encode_frames(frames[t % nslots].reshape(-1), None, sp["rec"], sp["li"], width=w, height=h,
                              intra=True, quant=args.quant, out=sp["out"])

    for t in range(args.warmup):
        step(t)
    elapsed, kavg, clk = timed_region(torch, dist, world, args.steps, args.warmup, step,
                                      graph=not args.eager, spinup_ms=args.spinup_ms,
                                      spin={"init": spin_init, "reset": spin_reset, "launch": spin_step})
    sp.clear()
    tmax = max_over_ranks(elapsed, world, device="cuda")
    last = args.warmup + args.steps - 1
    verified = None
    if not args.no_verify:
        import oracle
        coef, mb, _, recon = oracle.encode_sequence([frames[last % nslots, 0].cpu().numpy()], w, h,
                                                    quant=args.quant)[0]
        verified = bool(np.array_equal(out.coef[0].cpu().numpy(), coef)
                        and np.array_equal(out.mb[0].cpu().numpy().view(p64_amd.MB_DTYPE)
                                           .reshape(nmb), mb)
                        and np.array_equal(rec[:pic].cpu().numpy(), recon))
    if not all_ranks_ok(verified is not False, world, device="cuda"):
        raise SystemExit("bench: intra output differs from the oracle -- refusing to report")
    mbs = S * nmb
    key = content_key(args, f"{w}x{h}_intra_q{args.quant}_S{S}")
    return {"metric": METRICS["intra"], "value": round(aggregate_rate(world, mbs, args.steps, tmax), 1),
            "ms_per_step": round(tmax / args.steps * 1e3, 4),
            "config": {"workload": f"{w}x{h} intra pictures, q={args.quant}, content {args.content}, "
                                   f"{S} pictures/step/GPU", "macroblocks_per_step_per_gpu": mbs,
                       "distinct_input_pictures": nslots},
            "roofline": roofline(mbs * INTRA_BYTES_PER_MB, kavg,
                                 intra_kernel_name(args.quant),
                                 load_pmc(args.pmc_json, key),
                                 algorithmic_bytes_per_mb=INTRA_BYTES_PER_MB, timing=timing_note(args)),
            "valu_busy": (load_pmc(args.pmc_json, key) or {}).get("valu_busy"),
            "valu_busy_note": VALU_BUSY_NOTE,
            "steady_state": clk,
            "verified_vs_oracle": verified}


def encode_all(args, torch, p64_amd, frames, S, nmb, pic, nslots, mode):
    """The decode config's input: every step's levels and records of an
    encoded closed-loop run (FULL search), kept resident."""
    w, h = args.width, args.height
    nsteps = 1 + args.warmup + args.steps
    ncoef = min(nsteps, nslots)
    coef_all = torch.empty((ncoef, S, nmb, 6, 64), dtype=torch.int16, device="cuda")
    mb_all = torch.empty((ncoef, S, nmb, 4), dtype=torch.int8, device="cuda")
    rec = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(2)]
    li = torch.zeros(S * nmb, dtype=torch.uint8, device="cuda")
    for t in range(nsteps):
        o = p64_amd.FrameBatchOut(coef=coef_all[t % ncoef], mb=mb_all[t % ncoef], me=None)
        p64_amd.encode_frames(frames[t % nslots].reshape(-1), rec[(t + 1) % 2], rec[t % 2], li,
                              width=w, height=h, intra=(t == 0), quant=args.quant, me_mode=mode,
                              search_limit=args.search_limit, out=o)
    torch.cuda.synchronize()
    return {"coef": coef_all, "mb": mb_all, "recon_last": rec[(nsteps - 1) % 2], "last": nsteps - 1}


def run_decode(args, torch, dist, np, p64_amd, world, enc, S, nmb, pic):
    """configs[4]: decoder reconstruction of every encoded picture in order
    (closed loop from the decoded picture 0); the last decoded picture must equal
    the encoder's reconstruction of it, for every sequence.  The levels go to
    the decoder PACKED (p64gpu_decode_recon_packed, ABI v3: the transmitted
    blocks only + a per-64-block index, what p64s_pack_levels makes of the
    host reader's output; built here on the device from the encoder's levels,
    outside the timed region) -- the line's kernel is k_recon_pk; the dense
    entry (k_recon_mbg) is timed the same way beside it (`dense`)."""
    w, h = args.width, args.height
    ncoef = enc["coef"].shape[0]
    last = enc["last"]
    if last + 1 > ncoef:  # levels of early steps were overwritten: cannot decode from 0
        return {"metric": METRICS["decode"], "value": None, "ms_per_step": None,
                "error": f"decode needs all {last + 1} steps' levels resident (MAX_SLOTS {ncoef})"}
    qmb = torch.full((S * nmb,), args.quant, dtype=torch.uint8, device="cuda")
    mask = torch.ones(S * nmb, dtype=torch.uint8, device="cuda")
    first = last - args.steps + 1
    # the packed layout of every picture (the reader's job in a decoder)
    # (every picture's levels in one buffer, as a reader filling a batch
    # would: separately allocated per picture they measured up to 2 us
    # apart run to run)
    pk, parts = {}, []
    for t in range(last + 1):
        lv, n, ix = p64_amd.pack_levels_device(enc["coef"][t], enc["mb"][t], mask, w, h)
        parts.append((lv, n, ix))
    lv_all = torch.zeros((max(1, sum(n for _, n, _ in parts)), 64), dtype=torch.int16, device="cuda")
    off = 0
    for t, (lv, n, ix) in enumerate(parts):
        if n:
            lv_all[off:off + n].copy_(lv)
        pk[t] = (lv_all[off:] if n else lv_all[:1], n, ix)
        off += n
    del parts
    nbytes = []
    ngr = (S * 6 * nmb + 63) // 64  # the index: 16 bytes per 64 blocks of the batch
    for t in range(first, last + 1):
        nbytes.append(decode_bytes(torch, enc["mb"][t], S * nmb) + 16 * ngr)

    def measure(packed):
        dec = [torch.zeros(S * pic, dtype=torch.uint8, device="cuda") for _ in range(2)]

        def dec_step(t, d=dec):
            if packed:
                lv, n, ix = pk[t]
                p64_amd.decode_recon_packed(d[(t + 1) % 2], d[t % 2], lv, n, ix, enc["mb"][t], qmb, mask,
                                            width=w, height=h)
            else:
                p64_amd.decode_recon(d[(t + 1) % 2], d[t % 2], enc["coef"][t], enc["mb"][t], qmb, mask,
                                     width=w, height=h)

        for t in range(first):  # pictures before the timed ones, untimed
            dec_step(t)
        sp = {}

        def spin_init():
            sp["dec"] = [torch.empty_like(d) for d in dec]

        def spin_reset():
            for a, b in zip(sp["dec"], dec):
                a.copy_(b)

        elapsed, kavg, clk = timed_region(torch, dist, world, args.steps, first, dec_step, graph=not args.eager,
                                          spinup_ms=args.spinup_ms,
                                          spin={"init": spin_init, "reset": spin_reset,
                                                "launch": lambda t: dec_step(t, sp["dec"])})
        sp.clear()
        ok = bool(torch.equal(dec[last % 2], enc["recon_last"]))
        return elapsed, kavg, clk, ok

    if os.environ.get("P64_DECODE_DENSE_FIRST", "0") != "0":  # (diagnostic: order effects)
        d_el, d_kavg, _, d_ok = measure(False)
        elapsed, kavg, clk, ok = measure(True)
    else:
        elapsed, kavg, clk, ok = measure(True)
        d_el, d_kavg, _, d_ok = measure(False)
    tmax = max_over_ranks(elapsed, world, device="cuda")
    if not all_ranks_ok(ok and d_ok, world, device="cuda"):
        raise SystemExit("bench: decoded pictures differ from the encoder's reconstruction")
    mbs = S * nmb
    bpl = sum(nbytes) / len(nbytes)
    key = content_key(args, f"{w}x{h}_decode_q{args.quant}_S{S}")
    return {"metric": METRICS["decode"], "value": round(aggregate_rate(world, mbs, args.steps, tmax), 1),
            "ms_per_step": round(tmax / args.steps * 1e3, 4),
            "config": {"workload": f"{w}x{h} decoder reconstruction of a GPU-encoded stream "
                                   f"(FULL SL={args.search_limit}, q={args.quant}, content "
                                   f"{args.content}), {S} sequences/GPU, closed loop, packed levels "
                                   f"(p64gpu_decode_recon_packed)",
                       "macroblocks_per_step_per_gpu": mbs},
            "roofline": roofline(bpl, kavg, "k_recon_pk", load_pmc(args.pmc_json, key),
                                 algorithmic_bytes_per_mb=round(bpl / mbs, 1), timing=timing_note(args)),
            "dense": {"kernel": "k_recon_mbg (p64gpu_decode_recon, dense levels)",
                      "kernel_avg_us": round(d_kavg * 1e6, 2),
                      "frac": round(bpl / d_kavg / 1e9 / HBM_PEAK_GBS, 4),
                      "macroblocks_per_s": round(aggregate_rate(world, mbs, args.steps, d_el), 1)},
            "valu_busy": (load_pmc(args.pmc_json, key) or {}).get("valu_busy"),
            "valu_busy_note": VALU_BUSY_NOTE,
            "steady_state": clk,
            "verified_vs_encoder": {"ok": ok and d_ok, "note": "last decoded picture == encoder "
                                                               "reconstruction, all sequences (both entries)"}}


def dry_main(args, rank, world):
    """Device-less stand-in of the timed region (tests of the launcher, the
    sharding and the reductions on a CPU box): gloo, a host step per picture.
    The line has the shape of a real one (contract keys, config, ranks)."""
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ranks = rank_info(world, rank, local, dist)
    seed0, S = shard_seeds(rank, args.streams)
    nmb = (args.width // 16) * (args.height // 16)
    t0 = time.perf_counter()
    if world > 1:
        dist.barrier()
    for _ in range(args.steps):
        time.sleep(0.001 * (1 + rank))  # rank r is slower: the MAX must see it
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tmax = max_over_ranks(elapsed, world)
    seeds = [seed0, seed0 + S - 1]
    allseeds = seeds
    if world > 1:
        import torch
        t = torch.tensor(seeds, dtype=torch.int64)
        g = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(g, t)
        allseeds = torch.stack(g).tolist()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"metric": METRICS[args.config], "value": aggregate_rate(world, S * nmb, args.steps, tmax),
                          "unit": "macroblocks/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": tmax / args.steps * 1e3,
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                          "dtype": "u8", "data": "dry run (no device)",
                          "config": {"workload": "dry", "sequences_per_gpu": S,
                                     "macroblocks_per_step_per_gpu": S * nmb},
                          "dry": True, "elapsed_max_s": tmax, "seed_ranges": allseeds,
                          "ranks": ranks}), flush=True)


if __name__ == "__main__":
    main()
