#!/usr/bin/env python3
"""LLaMA-7B SpecInfer (LLaMA-68M SSM) decoded tokens/s on MI355X.

Workload (BASELINE.json metric / SURVEY.md §8d): 8 requests, prompt = BOS +
127 ids (splitmix64, seed 20250117), 128 decoded tokens each (max_length
256), max_tokens_per_batch 1024, max_spec_tree_token_num 23, tree widths
(1,1,3), 8 SSM steps per verify; synthetic seeded weights (no checkpoints
offline).  One "step" = one generate() of the whole 8-request batch.
N GPUs = tensor parallelism over N ranks (one process per GPU, RCCL), the SSM
replicated per rank.  value = decoded tokens of all requests / wall time
(max over ranks).

The process never imports torch (torch bundles a second copy of the HIP
runtime); the multi-rank control plane (unique-id broadcast, barrier,
max-reduce of times) is a small TCP exchange on 127.0.0.1.
"""
import argparse
import json
import os
import socket
import statistics
import struct
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

fa = None  # flexflow_amd, imported by the rank processes only (after the launcher)
CTRL_TIMEOUT_S = 600  # a control-plane peer silent this long is dead: fail, never hang

LLAMA_7B = dict(num_layers=32, vocab_size=32000, num_heads=32, num_kv_heads=32, hidden=4096,
                intermediate=11008, rms_eps=1e-6, rope_theta=10000.0)
LLAMA_65B = dict(num_layers=80, vocab_size=32000, num_heads=64, num_kv_heads=64, hidden=8192,
                 intermediate=22016, rms_eps=1e-5, rope_theta=10000.0)
LLAMA_68M = dict(num_layers=2, vocab_size=32000, num_heads=12, num_kv_heads=12, hidden=768,
                 intermediate=3072, rms_eps=1e-6, rope_theta=10000.0)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
M64 = (1 << 64) - 1


def splitmix64_stream(seed):
    x = seed & M64
    while True:
        x = (x + 0x9E3779B97F4A7C15) & M64
        z = x
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        yield z ^ (z >> 31)


def make_prompts(n, length, vocab, seed=20250117):
    g = splitmix64_stream(seed)
    return [[3 + next(g) % (vocab - 3) for _ in range(length)] for _ in range(n)]


class Ctrl:
    """Rank-0-hub TCP control plane (bytes broadcast, barrier, max)."""

    def __init__(self, rank, world, port, timeout=CTRL_TIMEOUT_S):
        self.rank, self.world = rank, world
        self.peers = []
        if world == 1:
            return
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind(("127.0.0.1", port))
            srv.listen(world)
            srv.settimeout(timeout)  # a peer that never connects -> socket.timeout
            byrank = {}
            for _ in range(world - 1):
                c, _ = srv.accept()
                c.settimeout(timeout)
                byrank[struct.unpack("<I", self._recv(c, 4))[0]] = c
            srv.close()
            self.peers = [byrank[r] for r in sorted(byrank)]  # rank order
        else:
            deadline = time.time() + timeout
            while True:
                try:
                    self.sock = socket.create_connection(("127.0.0.1", port), timeout=timeout)
                    break
                except OSError:
                    if time.time() > deadline:
                        raise
                    time.sleep(0.2)
            self.sock.settimeout(timeout)
            self.sock.sendall(struct.pack("<I", rank))

    @staticmethod
    def _recv(s, n):
        b = b""
        while len(b) < n:
            chunk = s.recv(n - len(b))
            if not chunk:
                raise ConnectionError("control plane closed")
            b += chunk
        return b

    def bcast(self, data: bytes) -> bytes:
        if self.world == 1:
            return data
        if self.rank == 0:
            for p in self.peers:
                p.sendall(struct.pack("<I", len(data)) + data)
            return data
        n = struct.unpack("<I", self._recv(self.sock, 4))[0]
        return self._recv(self.sock, n)

    def max(self, v: float) -> float:
        if self.world == 1:
            return v
        if self.rank == 0:
            vals = [v] + [struct.unpack("<d", self._recv(p, 8))[0] for p in self.peers]
            m = max(vals)
            for p in self.peers:
                p.sendall(struct.pack("<d", m))
            return m
        self.sock.sendall(struct.pack("<d", v))
        return struct.unpack("<d", self._recv(self.sock, 8))[0]

    def barrier(self):
        self.max(0.0)

    def allgather(self, data: bytes):
        """Every rank's bytes, in rank order, on every rank."""
        if self.world == 1:
            return [data]
        if self.rank == 0:
            parts = [data]
            for p in self.peers:
                n = struct.unpack("<I", self._recv(p, 4))[0]
                parts.append(self._recv(p, n))
            blob = b"".join(struct.pack("<I", len(x)) + x for x in parts)
            self.bcast(blob)
        else:
            self.sock.sendall(struct.pack("<I", len(data)) + data)
            blob = self.bcast(b"")
        out, off = [], 0
        while off < len(blob):
            n = struct.unpack("<I", blob[off:off + 4])[0]
            out.append(blob[off + 4:off + 4 + n])
            off += 4 + n
        return out


def stdout_to_stderr(fn):
    """Run fn with file descriptor 1 pointed at stderr: RCCL prints a version
    banner on stdout at communicator creation, and stdout must carry only
    rank 0's JSON line."""
    import ctypes
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        return fn()
    finally:
        ctypes.CDLL(None).fflush(None)
        os.dup2(saved, 1)
        os.close(saved)


def device_sync():
    import ctypes
    h = ctypes.CDLL("libamdhip64.so.7")
    assert h.hipDeviceSynchronize() == 0


def run_generate(rm, llm, prompts, max_length, spec):
    res = fa.generate(rm, llm, prompts, max_length=max_length, spec=spec)
    new = sum(len(r.output_tokens) - len(r.input_tokens) for r in res)
    lat = [(r.latency_us / max(1, len(r.output_tokens) - len(r.input_tokens))) for r in res]
    return new, lat, res


def cpu_baseline(acceptance=1.0, prompt_len=128, batch=8, budget_s=12.0, incr_budget_s=8.0):
    """The CPU restatement (oracle/, test infrastructure) timed on the host,
    on a bounded sample of the same workload (the headline's metric first):
    - SpecInfer: LLaMA-7B verify steps (8 requests x 21-token trees at the
      GPU run's decode positions 128+: 168 tokens per step, the dense layers
      batched over them, orc_model_forward_multi) and, per verify, the
      LLaMA-68M SSM's 8 beam steps (tree layers of 1, 1, 3, ... tokens per
      request, widths (1,1,3)); tokens/s = batch x acceptance / (verify + its
      8 SSM steps), with the GPU run's own measured acceptance (tokens
      committed per request per verify), so both sides decode at the same
      rate of tokens per step;
    - incremental decoding: batched T = 8 decode steps (orc_model_decode_batch).
    The 128-token prefill is not run (~7 TMAC, minutes on the host): the
    first prompt_len KV rows hold zeros, so this is a timing sample (every
    step reads as many keys as the GPU run's), not a token replay."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    tree = 21  # 1 root + layers 1, 1, 3 x 6 (widths (1,1,3), 8 SSM steps)
    layer_sizes = [1, 1, 3, 3, 3, 3, 3, 3]
    m = O.Model(LLAMA_7B, 20250117, fp16=1, max_requests=batch, max_seq=prompt_len + 160)
    ssm = O.Model(LLAMA_68M, 68, fp16=1, max_requests=batch, max_seq=prompt_len + 160)
    g = splitmix64_stream(7)
    rnd = lambda n: [3 + next(g) % (LLAMA_7B["vocab_size"] - 3) for _ in range(n)]  # noqa: E731
    reqs = list(range(batch))
    t_verify, t_ssm, steps = 0.0, 0.0, 0
    t0 = time.time()
    while time.time() - t0 < budget_s and steps < 8:
        pos = prompt_len + steps  # one committed token per request per step
        t1 = time.time()
        depth = 0
        for k in layer_sizes:  # the SSM's beam steps build the tree layer by layer
            ssm.forward_multi(reqs, [k] * batch, [pos + depth] * batch, rnd(k * batch))
            depth += k
        t2 = time.time()
        m.forward_multi(reqs, [tree] * batch, [pos] * batch, rnd(tree * batch))
        t3 = time.time()
        t_ssm += t2 - t1
        t_verify += t3 - t2
        steps += 1
    spec = batch * acceptance * steps / (t_verify + t_ssm)
    # incremental decoding leg
    toks = rnd(batch)
    t0 = time.time()
    isteps = 0
    while isteps < 64 and time.time() - t0 < incr_budget_s:
        logits = m.decode_batch(reqs, toks, [prompt_len + isteps] * batch)
        toks = O.softmax_argmax(logits, fp16=1)[0].tolist()
        isteps += 1
    dti = time.time() - t0
    return dict(value=round(spec, 3), unit="decoded tokens/s",
                cores=int(O.lib().orc_num_threads()), kind="port",
                sample=(f"oracle LLaMA-7B SpecInfer with the LLaMA-68M SSM, batch {batch}: {steps} "
                        f"verify steps (168 tree tokens at positions {prompt_len}+) + "
                        f"{8 * steps} SSM beam steps, {t_verify + t_ssm:.1f}s "
                        f"(verify {t_verify / steps:.2f}s, SSM {t_ssm / (8 * steps) * 1e3:.1f}ms "
                        f"per step), at the GPU run's acceptance {acceptance:.3f} tokens per "
                        f"request per verify; prefill rows zero-filled, not computed"),
                verify_step_s=round(t_verify / steps, 3),
                ssm_step_ms=round(t_ssm / (8 * steps) * 1e3, 2),
                incr_decoding={"value": round(batch * isteps / dti, 3), "unit": "decoded tokens/s",
                               "sample": f"{isteps} batched decode steps at positions "
                                         f"{prompt_len}-{prompt_len + isteps - 1}, {dti:.1f}s"})


def run_leg(llm_cfg, ssm_cfg, prompts, max_len, B, mtb, rm_kw, args, widths, tree, seeds, ext,
            init):
    """One SpecInfer side leg (rank 0, one GPU): a warm and a timed generate
    of the headline's prompts with other tree widths / SSMs / weights."""
    kw = dict(rm_kw, max_spec_tree_token_num=tree)
    vt = mtb + tree * B
    llm = fa.Model(llm_cfg, "tree", max_requests=B, max_tokens=vt,
                   max_seq_len=kw["max_sequence_length"], max_tree_tokens=tree,
                   weight_seed=20250117, weights_folder=args.llm_weights, weight_init=init)
    ssms = [fa.Model(ssm_cfg, "beam", max_requests=B, max_tokens=vt,
                     max_seq_len=kw["max_sequence_length"], max_tree_tokens=tree, weight_seed=sd,
                     weights_folder=args.ssm_weights, weight_init=init) for sd in seeds]
    rm = fa.RequestManager(spec_tree_width=widths, spec_extensions=ext, **kw)
    for m in ssms:
        rm.register_ssm_model(m)
    run_generate(rm, llm, prompts, max_len, True)  # warm (graphs captured)
    device_sync()
    t = time.time()
    n, lat, _ = run_generate(rm, llm, prompts, max_len, True)
    device_sync()
    dt = time.time() - t
    st = rm.stats()
    llm.close()
    for m in ssms:
        m.close()
    return {"value": round(n / dt, 2), "unit": "tokens/s", "ms_per_generate": round(dt * 1e3, 1),
            "tree_widths": list(widths), "ssms": len(seeds), "max_spec_tree_token_num": tree,
            "weight_init": init,
            "tokens_per_request_verify": round(st.tokens_committed / max(1, st.request_verifies), 3),
            "tree_tokens_per_request_verify": round(st.tree_tokens_verified /
                                                    max(1, st.request_verifies), 2),
            "llm_steps_per_generate": st.llm_steps, "ssm_steps_per_generate": st.ssm_steps,
            "verify_step_ms": round(st.llm_us / 1e3 / max(1, st.llm_steps), 3),
            "ssm_step_us": round(st.ssm_us / max(1, st.ssm_steps), 1),
            "p50_token_latency_ms": round(statistics.median(lat) / 1000.0, 3)}


def pmc_traffic(kernel):
    """HBM bytes per launch of the roofline kernel, measured with rocprofv3
    --pmc FETCH_SIZE in a separate run (scripts/round_gpu.sh ->
    scripts/pmc_summary.py -> profiles/rNN_pmc_fetch.json); None if absent."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_fetch.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("kernel") == kernel:
            d["source"] = os.path.relpath(f, ROOT)
            return d
    return None


MID_GATE_UP = "ffmi::gemm_mid_kernel<3, 6, 4, 1, false, true>"


def pmc_mfma(hip_kernel):
    """MFMA utilisation (SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel
    cycles)) of one kernel from the separate rocprofv3 --pmc pass
    (scripts/mfma_summary.py -> profiles/rNN_pmc_mfma.json); None if absent."""
    import glob
    for f in reversed(sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_mfma.json")))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        for k in d.get("kernels", []):
            if k["kernel"] == hip_kernel.replace("void ", ""):
                return {"mfma_util": k["mfma_util"], "source": os.path.relpath(f, ROOT)}
    return None


def launch_ranks(argv, n):
    """`python bench.py --gpus N` with no RANK in the environment: start N
    rank processes of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*
    set, one GPU each) and exit with the worst status.  The launcher never
    touches the GPU itself (no HIP call, no exec): it only spawns, waits and
    kills.  Rank 0's stdout is ours (the JSON line); the others' go to
    stderr."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(os.environ.get("MASTER_PORT", port)))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=None if r == 0 else sys.stderr.fileno()))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0:
                    rc = rc or code
                    for q in pending:  # one rank died: the others would wait forever
                        q.kill()
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
    return rc if rc > 0 else (1 if rc else 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--mode", choices=["spec", "incr"], default="spec")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--prefill", type=int, default=128)
    ap.add_argument("--decode", type=int, default=128)
    ap.add_argument("--max-tokens-per-batch", type=int, default=1024)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-incr", action="store_true", help="skip the incr-decoding side run")
    ap.add_argument("--no-legs", action="store_true",
                    help="skip the side legs (tree width 4, 4 SSMs, token-chain acceptance)")
    ap.add_argument("--profile", type=int, default=1,
                    help="op profiling level of the sampled generates run AFTER the timed "
                         "ones (roofline, op breakdown); the timed region never profiles")
    ap.add_argument("--profile-generates", type=int, default=2,
                    help="untimed generates sampled for the op breakdown")
    ap.add_argument("--layers", type=int, default=0, help="override LLM layer count (debug)")
    ap.add_argument("--llm-weights", default=None,
                    help="reference-format checkpoint folder with config.json (default: "
                         "seeded synthetic LLaMA-7B)")
    ap.add_argument("--ssm-weights", default=None,
                    help="reference-format checkpoint folder of the SSM (default: synthetic 68M)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher + control plane only, no GPU (CPU test of the N-rank path)")
    ap.add_argument("--dry-run-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", args.gpus))
    local = int(os.environ.get("LOCAL_RANK", rank))
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE {world} != --gpus {args.gpus}")
    if world > 1:
        # single node: RCCL's bootstrap over loopback (the data path is
        # xGMI peer-to-peer); an interface the user set wins
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    port = int(os.environ.get("MASTER_PORT", 29500)) + 31
    if args.dry_run and rank == args.dry_run_fail_rank:
        sys.exit(3)  # (test hook: a rank that dies before the control plane)
    ctrl = Ctrl(rank, world, port)
    if args.dry_run:
        ctrl.barrier()
        t = ctrl.max(float(rank))
        g = ctrl.allgather(b"r%d" % rank)
        if rank == 0:
            print(json.dumps({"metric": "dry-run", "value": None, "n_gpus": world,
                              "max_over_ranks": t, "allgather": [x.decode() for x in g]}),
                  flush=True)
        return
    global fa
    import flexflow_amd  # loads libffmi (first HIP use is below)
    fa = flexflow_amd
    # FFMI_BENCH_DEVICE pins every rank to one device: a rehearsal of the
    # N-rank path on a one-GPU box (with FFMI_TP_TRANSPORT=xgmi-only, since
    # RCCL refuses two ranks on one GPU); timings are then not a scaling result
    fa.set_device(int(os.environ.get("FFMI_BENCH_DEVICE", local)))
    comm = None
    transport = "rccl"
    transport_reason = "FFMI_TP_TRANSPORT=rccl"
    mode_tp = os.environ.get("FFMI_TP_TRANSPORT", "xgmi")  # xgmi | rccl | xgmi-only
    if world > 1:
        if mode_tp == "xgmi-only":
            comm = fa.Comm.peer(world, rank)
        else:
            uid = ctrl.bcast(stdout_to_stderr(fa.Comm.unique_id) if rank == 0 else b"")
            comm = stdout_to_stderr(lambda: fa.Comm(uid, world, rank))
        if mode_tp in ("xgmi", "xgmi-only"):
            # the direct xGMI all-reduce: exchange buffers sized for the
            # largest step's [T][H] fp16 partial, handles all-gathered here
            hid = (fa.llama_config_from_hf(args.llm_weights) if args.llm_weights
                   else LLAMA_7B)["hidden"]
            cap_tokens = args.max_tokens_per_batch + 23 * args.batch + 16
            try:
                mine = comm.export(cap_tokens * hid * 2)
            except Exception as e:  # noqa: BLE001 -- reported, then agreed on below
                print(f"[bench] rank {rank}: xGMI export failed ({e})", file=sys.stderr)
                transport_reason = f"rank {rank}: xGMI export failed ({e})"
                mine = b""
            handles = ctrl.allgather(mine)
            ok = 0.0
            if all(handles):  # every rank exported: attach (collective self-test)
                try:
                    comm.attach(handles)
                    ok = 1.0
                except Exception as e:  # noqa: BLE001
                    print(f"[bench] rank {rank}: xGMI attach failed ({e})", file=sys.stderr)
                    transport_reason = f"rank {rank}: xGMI attach failed ({e})"
            elif mine:
                transport_reason = "another rank's xGMI export failed"
            if -ctrl.max(-ok) < 1.0:  # some rank failed: every rank stays on RCCL
                if mode_tp == "xgmi-only":
                    raise SystemExit("xGMI transport failed and FFMI_TP_TRANSPORT=xgmi-only")
                comm.detach()
                if transport_reason.startswith("FFMI"):
                    transport_reason = "another rank's xGMI attach failed"
                # every rank reports rank 0's view; the reason of the failing
                # rank is on that rank's stderr
            else:
                transport = "xgmi"
                transport_reason = "direct xGMI all-reduce attached on every rank"

    llm_cfg = fa.llama_config_from_hf(args.llm_weights) if args.llm_weights else dict(LLAMA_7B)
    ssm_cfg = fa.llama_config_from_hf(args.ssm_weights) if args.ssm_weights else dict(LLAMA_68M)
    if args.layers:
        llm_cfg["num_layers"] = args.layers
    B, P, D = args.batch, args.prefill, args.decode
    max_len = P + D
    mtb = args.max_tokens_per_batch
    tree = 23
    widths = (1, 1, 3)
    prompts = make_prompts(B, P - 1, llm_cfg["vocab_size"])  # + BOS = P tokens
    verify_cap = mtb + tree * B

    spec = args.mode == "spec"
    rm_kw = dict(max_requests_per_batch=B, max_tokens_per_batch=mtb,
                 max_spec_tree_token_num=tree, max_sequence_length=max(512, max_len + 1))
    t_init = time.time()
    if spec:
        llm = fa.Model(llm_cfg, "tree", max_requests=B, max_tokens=verify_cap,
                       max_seq_len=rm_kw["max_sequence_length"], max_tree_tokens=tree,
                       weight_seed=20250117, tp_rank=rank, tp_size=world, comm=comm,
                       weights_folder=args.llm_weights)
        ssm = fa.Model(ssm_cfg, "beam", max_requests=B, max_tokens=verify_cap,
                       max_seq_len=rm_kw["max_sequence_length"], max_tree_tokens=tree,
                       weight_seed=68, weights_folder=args.ssm_weights)
        rm = fa.RequestManager(spec_tree_width=widths, **rm_kw)
        rm.register_ssm_model(ssm)
    else:
        llm = fa.Model(llm_cfg, "inc", max_requests=B, max_tokens=mtb,
                       max_seq_len=rm_kw["max_sequence_length"], weight_seed=20250117,
                       tp_rank=rank, tp_size=world, comm=comm, weights_folder=args.llm_weights)
        rm = fa.RequestManager(**rm_kw)
    init_s = time.time() - t_init
    if os.environ.get("FFMI_DUMP_MAPS"):  # diagnostics: library layout of this process
        with open("/proc/self/maps") as f, open(os.environ["FFMI_DUMP_MAPS"], "w") as g:
            g.write(f.read())

    # every rank has built its models (weights generated or loaded, graphs
    # not yet) before the first collective: the xGMI all-reduce waits at most
    # FFMI_PEER_TIMEOUT_S for a peer, and loading skew must not eat into that
    device_sync()
    ctrl.barrier()

    def progress(msg):  # rank 0, stderr: a long run (N ranks) stays visibly alive
        if rank == 0:
            print(f"[bench] {msg} ({time.time() - t_init:.1f} s)", file=sys.stderr, flush=True)

    progress("models built")
    for i in range(args.warmup):
        run_generate(rm, llm, prompts, max_len, spec)
        progress(f"warmup {i + 1}/{args.warmup}")
    ctrl.barrier()
    device_sync()
    t0 = time.time()
    new_tokens, lats, llm_steps, ssm_steps = 0, [], 0, 0
    committed, req_verifies = 0, 0
    llm_us, ssm_us, wall_us = 0.0, 0.0, 0.0
    for _ in range(args.steps):
        n, lat, res = run_generate(rm, llm, prompts, max_len, spec)
        st = rm.stats()
        new_tokens += n
        lats += lat
        llm_steps += st.llm_steps
        ssm_steps += st.ssm_steps
        committed += st.tokens_committed
        req_verifies += st.request_verifies
        llm_us += st.llm_us
        ssm_us += st.ssm_us
        wall_us += st.wall_us
        progress(f"step {_ + 1}/{args.steps}")
    device_sync()
    ctrl.barrier()
    elapsed = ctrl.max(time.time() - t0)
    # op breakdown / roofline: sampled in extra generates after the timed
    # region (op profiling runs every 4th step eager with events around the
    # ops of layers 0 and L/2), so the timed steps run as in production
    ops = {}
    if args.profile and args.profile_generates > 0:
        llm.set_profiling(args.profile)
        for _ in range(args.profile_generates):
            run_generate(rm, llm, prompts, max_len, spec)
        device_sync()
        ops = llm.op_stats()
        llm.set_profiling(0)
        ctrl.barrier()
        progress(f"profiled {args.profile_generates} untimed generates")

    value = new_tokens / elapsed  # every rank decodes the same requests (TP)
    out = {
        "metric": "decoded tokens/s (LLaMA-7B SpecInfer, LLaMA-68M SSM)" if spec else
                  "decoded tokens/s (LLaMA-7B incremental decoding)",
        "value": round(value, 2), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 2),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f16",
        "data": ("synthetic prompts, checkpoint weights" if args.llm_weights else
                 "synthetic (seeded random weights and prompts)"),
        "config": {"workload": ("llama7b_specinfer_llama68m" if spec else "llama7b_incr") +
                   f"_b{B}_p{P}_d{D}",
                   "model": (f"LLaMA ({args.llm_weights})" if args.llm_weights
                             else "LLaMA-7B (random init)"),
                   "ssm": ((f"LLaMA ({args.ssm_weights})" if args.ssm_weights
                            else "LLaMA-68M (random init)") if spec else None),
                   "global_batch": B, "prefill": P, "decode": D, "seq_len": max_len,
                   "parallelism": f"tp{world}",
                   "tp_transport": transport if world > 1 else None,
                   "tp_transport_reason": transport_reason if world > 1 else None,
                   "tree_widths": list(widths) if spec else None,
                   "max_tokens_per_batch": mtb, "layers": llm_cfg["num_layers"]},
        "p50_token_latency_ms": round(statistics.median(lats) / 1000.0, 3),
        "llm_steps_per_generate": llm_steps / args.steps,
        "ssm_steps_per_generate": ssm_steps / args.steps,
        "init_s": round(init_s, 1),
        # where a generate's wall time goes (host timers around the model steps)
        "time_split_ms_per_generate": {
            "llm_steps": round(llm_us / 1e3 / args.steps, 1),
            "ssm_steps": round(ssm_us / 1e3 / args.steps, 1),
            "host_scheduling": round((wall_us - llm_us - ssm_us) / 1e3 / args.steps, 1)},
    }
    if spec:
        # tokens each request commits per verify step (incl. the bonus token).
        # With random weights the SSM's guesses match at chance level, so this
        # is ~1.0: SpecInfer then pays a full verify step per token.  The
        # acceptance-independent step costs are reported beside it, and the
        # rate they imply at other acceptance levels is labelled a projection.
        acc = committed / max(1, req_verifies)
        out["acceptance"] = {"tokens_per_request_verify": round(acc, 3),
                             "note": "random weights: SSM agreement at chance level"}
        out["tokens_per_request_verify"] = round(acc, 3)
        verify_ms = llm_us / 1e3 / max(1, llm_steps)
        ssm_us_step = ssm_us / max(1, ssm_steps)
        out["verify_step_ms"] = round(verify_ms, 3)
        out["ssm_step_us"] = round(ssm_us_step, 1)
        cycle_ms = verify_ms + ssm_us_step / 1e3 * (ssm_steps / max(1, llm_steps))
        out["projection_tokens_per_s_at_acceptance"] = {
            str(a): round(B * a / (cycle_ms / 1e3), 1) for a in (1, 2, 3, 4)}
        out["projection_note"] = ("decode-phase rate B*a/(verify step + its SSM steps) from the "
                                  "measured step costs; not a measurement")
    # roofline of the dominant kernel: the weight-streaming GEMM with the
    # largest sampled time (HIP events on the model stream, timed region)
    gemms = {k: v for k, v in ops.items() if k.startswith("gemm") and v["ms"] > 0}
    if gemms:
        k = max(gemms, key=lambda x: gemms[x]["ms"])
        g = gemms[k]
        ach = g["bytes"] / (g["ms"] * 1e-3) / 1e9
        out["roofline"] = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                           "kernel": k, "launches_sampled": g["launches"],
                           "sampled_in": f"{args.profile_generates} untimed generates after "
                                         f"the timed region (HIP events on the model stream)",
                           "avg_launch_us": round(1000 * g["ms"] / g["launches"], 2),
                           "bytes_per_launch": round(g["bytes"] / g["launches"])}
        tr = pmc_traffic(k)
        if tr:
            out["roofline"]["traffic"] = tr["fetch_bytes_per_launch"]
            out["roofline"]["traffic_source"] = tr["source"]
            mf = pmc_mfma(tr.get("hip_kernel", MID_GATE_UP))
            if mf:
                out["roofline"]["mfma_util"] = mf["mfma_util"]
                out["roofline"]["mfma_util_source"] = mf["source"]
        out["op_breakdown_sampled"] = {
            kk: {"avg_us": round(1000 * v["ms"] / v["launches"], 2),
                 "GBps": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1) if v["ms"] else None,
                 "launches": v["launches"]} for kk, v in ops.items()}
    if rank == 0 and world == 1 and spec and not args.no_incr:
        inc = fa.Model(llm_cfg, "inc", max_requests=B, max_tokens=mtb,
                       max_seq_len=rm_kw["max_sequence_length"], weight_seed=20250117,
                       weights_folder=args.llm_weights)
        rmi = fa.RequestManager(**rm_kw)
        run_generate(rmi, inc, prompts, max_len, False)  # warm
        t1 = time.time()
        n, lat, _ = run_generate(rmi, inc, prompts, max_len, False)
        dt = time.time() - t1
        out["incr_decoding"] = {"value": round(n / dt, 2), "unit": "tokens/s",
                                "p50_token_latency_ms": round(statistics.median(lat) / 1000, 3),
                                "llm_steps": rmi.stats().llm_steps}
        inc.close()
    if rank == 0 and world == 1 and spec and not args.no_legs:
        # side legs, one warm + one timed generate each, same prompts and
        # lengths as the headline (BASELINE configs C / E as stated, and
        # SpecInfer at the acceptance a trained SSM gives):
        #  spec_width4      widths (1,1,4), 27-token trees (FFMI_SPEC_EXT_WIDTH4)
        #  spec_4ssm        4 LLaMA-68M SSMs (seeds 68-71), merged trees <= 64
        #                   tokens (FFMI_SPEC_EXT_MULTI_SSM)
        #  spec_token_chain widths (1,1,3), both models in the token-chain
        #                   synthetic init (include/ffmi.h): the SSM predicts
        #                   the LLM's greedy chain, so verify steps commit deep
        #                   paths (tree_inc_multihead_self_attention.cu:335-396)
        legs = {"spec_width4": dict(widths=(1, 1, 4), tree=27, seeds=(68,),
                                    ext=fa.ffmi.SPEC_EXT_WIDTH4, init="uniform"),
                "spec_4ssm": dict(widths=(1, 1, 3), tree=64, seeds=(68, 69, 70, 71),
                                  ext=fa.ffmi.SPEC_EXT_MULTI_SSM, init="uniform"),
                "spec_token_chain": dict(widths=(1, 1, 3), tree=23, seeds=(68,), ext=0,
                                         init="token_chain")}
        llm.close()  # free the headline model's 13.5 GB first
        llm = None
        for name, lg in legs.items():
            out[name] = run_leg(llm_cfg, ssm_cfg, prompts, max_len, B, mtb, rm_kw, args, **lg)
            progress(f"leg {name}: {out[name]['value']} tokens/s")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(
            acceptance=out.get("tokens_per_request_verify", 1.0) if spec else 1.0)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if llm is not None:
        llm.close()
    if comm:
        comm.close()


if __name__ == "__main__":
    main()
