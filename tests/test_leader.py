"""Lease-based leader election against the in-process fake API server
(reference: cmd/tf-operator.v1/app/server.go:55-59,168-193 -- one leader
out of N, failover after the lease expires, OnStoppedLeading stops the
process; the ``tf_operator_is_leader`` gauge, server.go:64-69)."""
import asyncio
import datetime
import urllib.request

from tf_operator_amd.fakeapi.server import FakeAPIServer
from tf_operator_amd.operator.kube import KubeClient
from tf_operator_amd.operator.leader import LeaderElector
from tf_operator_amd.operator.main import Operator, parse_args

FAST = dict(lease_duration=1.0, renew_deadline=0.5, retry_period=0.1)
LEASE = "coordination.k8s.io/leases"


async def _until(pred, timeout=10.0, interval=0.02):
    t = asyncio.get_running_loop().time() + timeout
    while asyncio.get_running_loop().time() < t:
        if pred():
            return True
        await asyncio.sleep(interval)
    return False


def _run(coro):
    return asyncio.run(asyncio.wait_for(coro, 60))


def test_one_leader_then_failover_after_lease_expiry():
    async def main():
        api = FakeAPIServer()
        url = await api.start()
        kube = KubeClient(url, qps=0)
        events = []
        stops = [asyncio.Event(), asyncio.Event()]
        els = [LeaderElector(kube, "kubeflow", "tf-operator", identity=f"op-{i}",
                             on_started=lambda i=i: events.append(("start", i)),
                             on_stopped=lambda i=i: events.append(("stop", i)), **FAST) for i in range(2)]
        tasks = [asyncio.create_task(e.run(s)) for e, s in zip(els, stops)]
        assert await _until(lambda: any(e.is_leader for e in els))
        await asyncio.sleep(0.5)  # several retry periods: the other one must stay a follower
        leaders = [i for i, e in enumerate(els) if e.is_leader]
        assert len(leaders) == 1, leaders
        first = leaders[0]
        lease = await kube.get(LEASE, "kubeflow", "tf-operator")
        assert lease["spec"]["holderIdentity"] == f"op-{first}"
        assert lease["spec"]["leaseDurationSeconds"] == 1
        # the leader process dies without releasing the lease
        tasks[first].cancel()
        t_dead = asyncio.get_running_loop().time()
        other = 1 - first
        assert await _until(lambda: els[other].is_leader, timeout=5)
        took = asyncio.get_running_loop().time() - t_dead
        assert took >= 0.5, took  # not before the lease could have expired (renewed within the last retry)
        lease = await kube.get(LEASE, "kubeflow", "tf-operator")
        assert lease["spec"]["holderIdentity"] == f"op-{other}"
        assert lease["spec"]["leaseTransitions"] == 1
        assert ("start", other) in events
        stops[other].set()
        await asyncio.gather(tasks[other], return_exceptions=True)
        await kube.close()
        await api.stop()

    _run(main())


def test_leader_stops_when_lease_is_taken():
    """A leader that cannot renew (another holder with a fresh renewTime)
    gives up after renew_deadline and runs OnStoppedLeading."""
    async def main():
        api = FakeAPIServer()
        url = await api.start()
        kube = KubeClient(url, qps=0)
        stopped = asyncio.Event()
        el = LeaderElector(kube, "kubeflow", "tf-operator", identity="op-a", on_stopped=stopped.set, **FAST)
        task = asyncio.create_task(el.run())
        assert await _until(lambda: el.is_leader)

        async def usurp():  # keep the lease renewed under another identity
            while not stopped.is_set():
                lease = await kube.get(LEASE, "kubeflow", "tf-operator")
                lease["spec"]["holderIdentity"] = "op-b"
                lease["spec"]["renewTime"] = datetime.datetime.now(datetime.timezone.utc).strftime(
                    "%Y-%m-%dT%H:%M:%S.%fZ")
                try:
                    await kube.update(LEASE, "kubeflow", lease)
                except Exception:
                    pass
                await asyncio.sleep(0.05)

        u = asyncio.create_task(usurp())
        assert await _until(stopped.is_set, timeout=5)
        assert not el.is_leader
        await asyncio.gather(task, u, return_exceptions=True)
        await kube.close()
        await api.stop()

    _run(main())


def _gauge(port):
    body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
    for line in body.splitlines():
        if line.startswith("tf_operator_is_leader "):
            return float(line.split()[1])
    return None


def test_operator_is_leader_gauge_and_exit_on_loss():
    """--leader-elect: the gauge reads 1 while leading and /readyz turns
    ready; losing the lease sets it to 0 and stops the operator (the
    reference log.Fatalf's, server.go:186-188)."""
    async def main():
        api = FakeAPIServer()
        url = await api.start()
        args = parse_args(["--master", url, "--leader-elect", "--metrics-bind-address", "127.0.0.1:0",
                           "--health-probe-bind-address", "127.0.0.1:0", "--monitoring-port", "0",
                           "--leader-lease-duration", "1", "--leader-renew-deadline", "0.5",
                           "--leader-retry-period", "0.1", "--qps", "0"])
        assert parse_args([]).monitoring_port == 8443  # options.go:75 default
        op = Operator(args)
        run = asyncio.create_task(op.run())
        assert await _until(lambda: "metrics" in op.ports and op.ready, timeout=10)
        loop = asyncio.get_running_loop()
        assert await loop.run_in_executor(None, _gauge, op.ports["metrics"]) == 1.0
        kube = KubeClient(url, qps=0)
        # another instance takes the lease and keeps it fresh
        done = asyncio.Event()

        async def usurp():
            while not done.is_set():
                try:
                    lease = await kube.get(LEASE, "default", args.leader_election_id)
                    lease["spec"]["holderIdentity"] = "other-instance"
                    lease["spec"]["renewTime"] = datetime.datetime.now(datetime.timezone.utc).strftime(
                        "%Y-%m-%dT%H:%M:%S.%fZ")
                    await kube.update(LEASE, "default", lease)
                except Exception:
                    pass
                await asyncio.sleep(0.05)

        u = asyncio.create_task(usurp())
        assert await _until(op.stop.is_set, timeout=10)
        assert op.metrics.is_leader._value.get() == 0.0
        done.set()
        await asyncio.wait_for(run, 20)
        await u
        await kube.close()
        await api.stop()

    _run(main())
