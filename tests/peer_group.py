"""Run N rank processes of the direct xGMI transport on this machine's GPU(s).

Each rank is a fresh `spawn` process (no torch, no inherited HIP state) that
creates a peer communicator, exports its exchange buffer, receives every
rank's handle from the parent (the control plane of bench.py, here a pipe),
attaches, runs a task and sends its result back.  On the one-GPU test box
every rank uses device 0: the ranks are separate processes with separate
address spaces exchanging through IPC-mapped buffers -- the same protocol,
flags, epochs and fences as across the xGMI links of an 8-GPU node, only the
bytes do not leave the device.  Used by the -m gpu tests only.
"""
import multiprocessing as mp
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _child(rank, n, conn, task, args, env, max_bytes, device):
    try:
        for k, v in env.items():  # None: leave the variable unset (HIP's default)
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import flexflow_amd as fa
        fa.set_device(device(rank) if callable(device) else device)
        comm = fa.Comm.peer(n, rank)
        conn.send(comm.export(max_bytes))
        handles = conn.recv()
        comm.attach(handles)
        res = task(fa, comm, rank, n, *args)
        if not getattr(comm, "expect_error", False):
            comm.status()
        conn.send(("ok", res))
        comm.close()
    except BaseException:  # noqa: BLE001 -- reported to the parent
        conn.send(("err", traceback.format_exc()))
    finally:
        conn.close()


def run_group(n, task, args=(), env=None, max_bytes=1 << 22, timeout=240, device=0):
    """Run task(fa, comm, rank, n, *args) on n ranks; returns [result per rank].
    A rank that fails, or a group that exceeds `timeout`, raises.

    Each rank gets GPU_MAX_HW_QUEUES=1 unless `env` says otherwise: n processes
    with HIP's default of up to 4 hardware queues each (their compute and
    all-reduce streams) oversubscribe the device's queue slots, the scheduler
    then time-slices between processes, and every all-reduce waits out the
    slices of the peers it spins on (8 ranks of the 7B bench: 370 s per
    generate; with one queue per rank 7.6 s).  One queue serialises a rank's
    two streams in issue order -- the cross-stream waits still hold, only the
    overlap is gone -- which changes no value.  env={"GPU_MAX_HW_QUEUES": None}
    keeps HIP's default (up to 4 queues per rank: compute and all-reduce streams
    overlap, the production setting of a one-process-per-GPU node)."""
    env = {"GPU_MAX_HW_QUEUES": "1", **(env or {})}
    ctx = mp.get_context("spawn")
    pipes, procs = [], []
    for r in range(n):
        a, b = ctx.Pipe()
        p = ctx.Process(target=_child, args=(r, n, b, task, args, env, max_bytes, device))
        p.start()
        pipes.append(a)
        procs.append(p)
    try:
        handles = []
        for r, c in enumerate(pipes):
            if not c.poll(timeout):
                raise TimeoutError(f"rank {r} never exported its handle")
            h = c.recv()
            if isinstance(h, tuple):
                raise RuntimeError(f"rank {r} failed before attach:\n{h[1]}")
            handles.append(h)
        for c in pipes:
            c.send(handles)
        out = []
        for r, c in enumerate(pipes):
            if not c.poll(timeout):
                raise TimeoutError(f"rank {r} did not finish in {timeout}s")
            st, res = c.recv()
            if st != "ok":
                raise RuntimeError(f"rank {r} failed:\n{res}")
            out.append(res)
        return out
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
                p.join()
