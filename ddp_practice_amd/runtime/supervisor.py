"""Rank supervisor: run a multi-rank program as FRESH child processes, detect a
failed or stalled attempt, and let the caller retry it with other settings.

The reference's launchers give failure handling to torch: ``mp.spawn`` joins
and re-raises the first child exception (/root/reference/ddp_main.py:173-178,
torch/multiprocessing/spawn.py:118-211), torchrun's agent tears the group down
(``max_restarts=0``), and ProcessGroupNCCL's watchdog bounds a stuck collective
(SURVEY.md §5).  None of them can run the SAME job again with a safer
communicator.  This module can, and it never re-executes a process that has
touched the GPU: every attempt is a new set of child processes started by a
parent that never initialises HIP (the supervisor only reads environment
variables, a TCPStore and the children's exit status / status files).

Two shapes, one protocol:

* self-launch (``python bench.py --gpus N``): one supervisor owns all N ranks;
* torchrun (``torchrun --nproc-per-node N bench.py``): every torchrun worker is
  the supervisor of ONE child rank; the supervisors agree through the torchrun
  agent's TCPStore (``MASTER_ADDR``/``MASTER_PORT``), so every one of them takes
  the same retry decision from the same gathered results.

Per attempt the leader (global rank 0's supervisor) hosts a fresh TCPStore for
the children's ``init_process_group(env://)`` rendezvous (children connect as
clients: ``TORCHELASTIC_USE_AGENT_STORE=True``), so attempts never share keys.
A child that exits non-zero raises a shared ``failed`` flag; every other child
then gets ``grace_s`` to finish on its own (its native watchdog usually reports
why first) before its process group is killed.  A whole attempt is bounded by
``timeout_s``.  Each child's stderr is streamed through (prefixed ``[rank r]``)
and its tail kept for the failure report.
"""
from __future__ import annotations

import collections
import datetime
import json
import os
import signal
import subprocess
import sys
import threading
import time
from dataclasses import dataclass, field


@dataclass
class RankResult:
    rank: int
    rc: int | None                       # None: killed by the supervisor (stall / peer failure)
    status: dict | None                  # the child's status file (None if it never wrote one)
    stderr_tail: list[str] = field(default_factory=list)
    killed: str = ""                     # why the supervisor killed it ("" if it exited itself)

    def to_json(self) -> dict:
        return {"rank": self.rank, "rc": self.rc, "status": self.status, "stderr_tail": self.stderr_tail,
                "killed": self.killed}

    @staticmethod
    def from_json(d: dict) -> "RankResult":
        return RankResult(d["rank"], d["rc"], d["status"], d.get("stderr_tail", []), d.get("killed", ""))

    @property
    def ok(self) -> bool:
        return self.rc == 0 and self.status is not None and not self.status.get("comm_error")

    def error(self) -> str:
        """One line: why this rank's attempt is not usable ("" if it is)."""
        if self.status is not None and self.status.get("comm_error"):
            return str(self.status["comm_error"])
        if self.rc == 0 and self.status is not None:
            return ""
        if self.killed:
            return self.killed
        why = ""
        for ln in reversed(self.stderr_tail):  # the native watchdog's report, else the last error line
            if "[dpa watchdog]" in ln:
                why = ln.strip()
                break
        if not why:
            for ln in reversed(self.stderr_tail):
                if any(k in ln for k in ("Error", "error", "Exception", "Traceback", "failed")):
                    why = ln.strip()
                    break
        if self.rc == 0:
            return f"exited 0 without a status file{': ' + why if why else ''}"
        return f"exit {self.rc}{': ' + why if why else ''}"


def _store_client(host: str, port: int, timeout_s: float = 900.0):
    from torch.distributed import TCPStore

    return TCPStore(host, port, None, False, datetime.timedelta(seconds=timeout_s))


def _store_master(timeout_s: float = 900.0):
    from torch.distributed import TCPStore

    return TCPStore("127.0.0.1", 0, None, True, datetime.timedelta(seconds=timeout_s), wait_for_workers=False)


class Supervisor:
    """``run(argv, env, tag)`` -> list[RankResult] for every global rank (same list on every
    supervisor).  ``argv``: the child command (``[sys.executable, script, ...]``)."""

    def __init__(self, world: int, local_ranks: list[int] | None = None, grace_s: float = 10.0,
                 timeout_s: float = 300.0, echo=None):
        self.world = world
        torchrun = local_ranks is None
        if torchrun:  # one supervisor per rank, started by torchrun
            lws = int(os.environ.get("LOCAL_WORLD_SIZE", world))
            if lws != world:
                # the children's per-attempt rendezvous store lives on the leader's localhost
                # (and the xGMI engine is single-node): a rank on another node could only time
                # out after 300 s and be reported as a communicator failure
                raise ValueError(f"the rank supervisor is single-node: LOCAL_WORLD_SIZE={lws} != "
                                 f"WORLD_SIZE={world} (multi-node torchrun is not supported)")
            self.rank = int(os.environ["RANK"])
            self.local_ranks = [self.rank]
            self.local_rank_of = {self.rank: int(os.environ.get("LOCAL_RANK", self.rank))}
            host, port = os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"])
            if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True" or self.rank != 0:
                self.store = _store_client(host, port)
            else:  # torchrun without an agent store: rank 0 serves it, as init_process_group would
                from torch.distributed import TCPStore

                self.store = TCPStore(host, port, None, True, datetime.timedelta(seconds=900),
                                      wait_for_workers=False)
            from torch.distributed import PrefixStore

            # a run id keeps the keys of two runs on one long-lived agent store apart
            self.store = PrefixStore(f"dpa_sup/{os.environ.get('TORCHELASTIC_RUN_ID', 'run')}/", self.store)
        else:  # self-launch: this process owns every rank
            self.rank = 0
            self.local_ranks = list(local_ranks)
            self.local_rank_of = {r: r for r in self.local_ranks}
            self.store = None
        self.leader = 0 in self.local_ranks
        self.grace_s, self.timeout_s = grace_s, timeout_s
        self.echo = echo if echo is not None else (lambda s: print(s, file=sys.stderr, flush=True))
        self._n = 0

    # ------------------------------------------------------------------ helpers
    def _shared_set(self, key: str, val: str) -> None:
        if self.store is not None:
            self.store.set(key, val)
        else:
            self._local[key] = val

    def _shared_has(self, key: str) -> bool:
        if self.store is not None:
            return self.store.check([key])
        return key in self._local

    def _spawn(self, r: int, argv: list[str], env: dict, port: int, status_dir: str, tag: str):
        e = dict(os.environ)
        e.update(env)
        for k in ("TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS", "GROUP_RANK", "ROLE_RANK"):
            e.pop(k, None)
        e.update(RANK=str(r), LOCAL_RANK=str(self.local_rank_of[r]), WORLD_SIZE=str(self.world),
                 LOCAL_WORLD_SIZE=str(e.get("LOCAL_WORLD_SIZE", self.world)), MASTER_ADDR="127.0.0.1",
                 MASTER_PORT=str(port), TORCHELASTIC_USE_AGENT_STORE="True", DPA_BENCH_CHILD="1",
                 DPA_STATUS_FILE=os.path.join(status_dir, f"rank{r}.json"), PYTHONUNBUFFERED="1")
        p = subprocess.Popen(argv, env=e, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                             start_new_session=True)  # own process group: killable as a whole
        tail: collections.deque = collections.deque(maxlen=40)

        def pump():
            for ln in p.stderr:
                tail.append(ln.rstrip("\n"))
                self.echo(f"[{tag} rank {r}] {ln.rstrip()}")

        th = threading.Thread(target=pump, daemon=True)
        th.start()
        return p, tail, th

    @staticmethod
    def _kill(p) -> None:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except (ProcessLookupError, PermissionError):
            pass

    # ------------------------------------------------------------------ one attempt
    def run(self, argv: list[str], env: dict | None = None, tag: str = "attempt",
            timeout_s: float | None = None) -> list[RankResult]:
        import tempfile

        self._n += 1
        k = self._n
        self._local: dict = {}
        timeout_s = self.timeout_s if timeout_s is None else timeout_s
        child_store = None
        if self.leader:
            child_store = _store_master()
            port = child_store.port
            if self.store is not None:
                self.store.set(f"a{k}/port", str(port))
        else:
            port = int(self.store.get(f"a{k}/port"))
        status_dir = tempfile.mkdtemp(prefix=f"dpa_{tag}_")
        procs = {r: self._spawn(r, argv, env or {}, port, status_dir, tag) for r in self.local_ranks}
        t0 = time.monotonic()
        killed: dict[int, str] = {}
        fail_seen_at = None
        while True:
            running = [r for r, (p, _, _) in procs.items() if p.poll() is None]
            for r, (p, _, _) in procs.items():
                if p.returncode not in (None, 0) and not self._shared_has(f"a{k}/failed"):
                    self._shared_set(f"a{k}/failed", str(r))
            if not running:
                break
            now = time.monotonic()
            if fail_seen_at is None and self._shared_has(f"a{k}/failed"):
                fail_seen_at = now
            if fail_seen_at is not None and now - fail_seen_at > self.grace_s:
                for r in running:
                    killed[r] = f"killed {self.grace_s:.0f} s after a peer rank failed"
                    self._kill(procs[r][0])
            elif now - t0 > timeout_s:
                for r in running:
                    killed[r] = f"killed: attempt exceeded {timeout_s:.0f} s (stalled)"
                    self._kill(procs[r][0])
                self._shared_set(f"a{k}/failed", "timeout")
            time.sleep(0.1)
        mine = []
        for r, (p, tail, th) in procs.items():
            p.wait()
            th.join(timeout=5)
            st = None
            path = os.path.join(status_dir, f"rank{r}.json")
            try:
                with open(path) as f:
                    st = json.load(f)
            except (OSError, ValueError):
                st = None
            mine.append(RankResult(r, None if r in killed else p.returncode, st, list(tail), killed.get(r, "")))
        results = self._gather(k, mine)
        del child_store
        return results

    def _gather(self, k: int, mine: list[RankResult]) -> list[RankResult]:
        if self.store is None:
            return sorted(mine, key=lambda x: x.rank)
        for m in mine:
            self.store.set(f"a{k}/res/{m.rank}", json.dumps(m.to_json()))
        keys = [f"a{k}/res/{r}" for r in range(self.world)]
        self.store.wait(keys, datetime.timedelta(seconds=self.timeout_s + 120))
        return [RankResult.from_json(json.loads(self.store.get(key))) for key in keys]


def summarize(results: list[RankResult]) -> str:
    """"" if every rank is usable, else one line naming each failing rank and why."""
    errs = [f"rank {r.rank}: {r.error()}" for r in results if not r.ok]
    return "; ".join(errs)
