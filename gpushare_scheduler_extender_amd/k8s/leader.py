"""Lease-based leader election (``coordination.k8s.io/v1`` Lease), client-go semantics.

High availability is a roadmap item of the reference (``README.md:79``): it
runs one replica with ``strategy: Recreate`` (``config/gpushare-schd-extender.yaml:69-71``)
and, because the policy is ``ignorable: false``, GPU-share pods cannot
schedule while that replica restarts.  With ``--leader-elect`` several
extender replicas run hot (informers + ledger warm); exactly one holds the
Lease and binds, the others report not-ready on ``/healthz`` so the Service
routes kube-scheduler to the leader, and refuse binds if they get one anyway.

Algorithm (``k8s.io/client-go/tools/leaderelection``): every ``retry_period``
try to create / renew the Lease with our identity; a Lease held by someone
else can be taken over only after ``lease_duration`` without the holder
renewing, measured on the *local* clock from when we last saw the record
change (clock skew between replicas does not matter).  A leader that cannot
renew within ``renew_deadline`` steps down.  All writes use the Lease's
resourceVersion, so two candidates can never both win.

Step-down is bounded like client-go's shared ``RenewDeadline`` context: a
renewal counts from the moment its attempt *started*, every attempt by the
leader is cut off at ``last_renew + renew_deadline`` (a hanging apiserver
call cannot stretch it), and the retry sleep never runs past that deadline.
So the old leader stops binding within ``renew_deadline`` of its last good
renewal, before a standby can take over (``lease_duration`` > ``renew_deadline``).
"""
from __future__ import annotations

import asyncio
import logging
import os
import socket
import time
import uuid
from datetime import datetime, timezone

from .client import ApiError, KubeClient

log = logging.getLogger("gsx.leader")


def _micro_time() -> str:
    return datetime.now(timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


class LeaderElector:
    def __init__(self, client: KubeClient, name: str = "gpushare-schd-extender", namespace: str = "kube-system",
                 identity: str | None = None, lease_duration: float = 15.0, renew_deadline: float = 10.0,
                 retry_period: float = 2.0, on_started=None, on_stopped=None):
        self.client = client
        self.name = name
        self.namespace = namespace
        self.identity = identity or f"{socket.gethostname()}_{os.getpid()}_{uuid.uuid4().hex[:6]}"
        self.lease_duration = lease_duration
        self.renew_deadline = renew_deadline
        self.retry_period = retry_period
        self.on_started = on_started
        self.on_stopped = on_stopped
        self.is_leader = False
        self.transitions = 0
        self._observed: tuple | None = None  # (holder, renewTime) last seen
        self._observed_at = 0.0
        self._last_renew = 0.0
        self._task: asyncio.Task | None = None
        self._stopping = False

    def _lease_obj(self, cur: dict | None) -> dict:
        now = _micro_time()
        spec = dict((cur or {}).get("spec") or {})
        if spec.get("holderIdentity") != self.identity:
            spec["acquireTime"] = now
            spec["leaseTransitions"] = int(spec.get("leaseTransitions") or 0) + (1 if cur else 0)
        spec.update({"holderIdentity": self.identity, "leaseDurationSeconds": int(self.lease_duration),
                     "renewTime": now})
        md = {"name": self.name, "namespace": self.namespace}
        if cur:
            md["resourceVersion"] = cur["metadata"]["resourceVersion"]
        return {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease", "metadata": md, "spec": spec}

    async def try_acquire_or_renew(self) -> bool:
        t0 = time.monotonic()  # a successful write happened after this: the conservative renewal time
        try:
            cur = await self.client.get("leases", self.name, self.namespace)
        except ApiError as e:
            if not e.not_found:
                raise
            try:
                await self.client.create("leases", self._lease_obj(None), self.namespace)
            except ApiError as e2:
                if e2.status == 409:
                    return False
                raise
            self._last_renew = t0
            return True
        spec = cur.get("spec") or {}
        holder = spec.get("holderIdentity") or ""
        rec = (holder, spec.get("renewTime"))
        now = time.monotonic()
        if rec != self._observed:
            self._observed, self._observed_at = rec, now
        duration = float(spec.get("leaseDurationSeconds") or self.lease_duration)
        if holder and holder != self.identity and now < self._observed_at + duration:
            return False  # someone else holds a live lease
        try:
            await self.client.replace("leases", self._lease_obj(cur))
        except ApiError as e:
            if e.conflict:
                return False
            raise
        self._last_renew = t0
        return True

    def _deadline_left(self) -> float:
        return self._last_renew + self.renew_deadline - time.monotonic()

    def _step_down(self):
        if self.is_leader:
            self.is_leader = False
            log.warning("%s lost leadership of %s/%s", self.identity, self.namespace, self.name)
            if self.on_stopped:
                self.on_stopped()

    async def _run(self):
        # The flag, not only the cancel, ends the loop: before Python 3.12 asyncio.wait_for returns the
        # inner result and swallows a cancellation that lands just as the inner call completes, and a
        # loop that relied on CancelledError alone would renew forever (stop() would never return).
        while not self._stopping:
            timeout = self.renew_deadline
            if self.is_leader:
                timeout = self._deadline_left()
                if timeout <= 0:
                    self._step_down()
                    timeout = self.renew_deadline
            try:
                ok = await asyncio.wait_for(self.try_acquire_or_renew(), timeout)
            except (ApiError, OSError, ConnectionError, asyncio.TimeoutError) as e:
                log.warning("lease %s/%s: %r", self.namespace, self.name, e)
                ok = False
            if ok and not self.is_leader:
                self.is_leader = True
                self.transitions += 1
                log.info("%s became leader of %s/%s", self.identity, self.namespace, self.name)
                if self.on_started:
                    self.on_started()
            elif not ok and self.is_leader and self._deadline_left() <= 0:
                self._step_down()
            sleep = self.retry_period
            if self.is_leader:
                sleep = max(0.0, min(sleep, self._deadline_left()))
            await asyncio.sleep(sleep)

    async def start(self):
        self._task = asyncio.get_running_loop().create_task(self._run(), name=f"leader-{self.name}")

    async def stop(self, release: bool = True):
        self._stopping = True
        if self._task:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
        if release and self.is_leader:
            # hand over immediately: an expired-looking lease (client-go ReleaseOnCancel)
            try:
                cur = await self.client.get("leases", self.name, self.namespace)
                if (cur.get("spec") or {}).get("holderIdentity") == self.identity:
                    cur["spec"]["holderIdentity"] = ""
                    cur["spec"]["leaseDurationSeconds"] = 1
                    await self.client.replace("leases", cur)
            except (ApiError, OSError, ConnectionError):
                pass
        if self.is_leader and self.on_stopped:
            self.on_stopped()
        self.is_leader = False
