"""Which GPU this replica drives, when it can see more than its own.

In the node-local layout (csrc/core/nodelocal.cc, annotation
``amd.com/node-local: privileged``) the training container is privileged so
that RCCL reaches its peers over xGMI -- and therefore sees EVERY GPU of the
node, including GPUs the device plugin gave to other jobs.  ``LOCAL_RANK``
does not name the pod's GPU then.  The kubelet does: its pod-resources API
(``/var/lib/kubelet/pod-resources/kubelet.sock``, gRPC
``v1.PodResourcesLister/List``) lists, per pod and container, the device IDs
allocated for each extended resource; the AMD device plugin's IDs for
``amd.com/gpu`` are the GPUs' PCI addresses.  :func:`allocated_device_index`
asks it for this pod's IDs and returns the HIP ordinal whose PCI address
matches.  Anything it cannot resolve raises: binding a guessed GPU on a shared
node would silently run on someone else's device.

The protobuf messages are decoded by hand (:func:`decode`, the 40 lines of
wire format the List response needs), so no generated stubs are required;
the transport is grpcio.

Reference anchor: the env contract the operator injects per replica
(pkg/controller.v1/pytorch/pytorch.go:40-65) and the reference's one-GPU-per-
worker layout (examples/v1/distribution_strategy/keras-API/
multi_worker_tfjob.yaml:19-21); device allocation itself is the kubelet's.
"""
from __future__ import annotations

import os
import re

SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"
LIST_METHOD = "/v1.PodResourcesLister/List"


# ---------------------------------------------------------------- protobuf
def _varint(b: bytes, i: int):
    shift = out = 0
    while True:
        c = b[i]
        i += 1
        out |= (c & 0x7F) << shift
        if c < 0x80:
            return out, i
        shift += 7


def fields(b: bytes):
    """Yield (field_number, wire_type, value) of one protobuf message
    (value: int for varint / fixed, bytes for length-delimited)."""
    i = 0
    while i < len(b):
        key, i = _varint(b, i)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(b, i)
        elif wt == 1:
            v, i = int.from_bytes(b[i:i + 8], "little"), i + 8
        elif wt == 2:
            n, i = _varint(b, i)
            v, i = b[i:i + n], i + n
        elif wt == 5:
            v, i = int.from_bytes(b[i:i + 4], "little"), i + 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield fn, wt, v


def decode(resp: bytes) -> list[dict]:
    """ListPodResourcesResponse -> [{name, namespace, containers: [{name,
    devices: [{resource_name, device_ids: [...]}]}]}]."""
    pods = []
    for fn, wt, v in fields(resp):
        if fn != 1 or wt != 2:
            continue
        pod = {"name": "", "namespace": "", "containers": []}
        for f2, w2, v2 in fields(v):
            if f2 == 1 and w2 == 2:
                pod["name"] = v2.decode()
            elif f2 == 2 and w2 == 2:
                pod["namespace"] = v2.decode()
            elif f2 == 3 and w2 == 2:
                c = {"name": "", "devices": []}
                for f3, w3, v3 in fields(v2):
                    if f3 == 1 and w3 == 2:
                        c["name"] = v3.decode()
                    elif f3 == 2 and w3 == 2:
                        d = {"resource_name": "", "device_ids": []}
                        for f4, w4, v4 in fields(v3):
                            if f4 == 1 and w4 == 2:
                                d["resource_name"] = v4.decode()
                            elif f4 == 2 and w4 == 2:
                                d["device_ids"].append(v4.decode())
                        c["devices"].append(d)
                pod["containers"].append(c)
        pods.append(pod)
    return pods


def _encode_str(fn: int, s: str) -> bytes:
    b = s.encode()
    return bytes([fn << 3 | 2]) + _enc_varint(len(b)) + b


def _enc_varint(n: int) -> bytes:
    out = bytearray()
    while True:
        c = n & 0x7F
        n >>= 7
        out.append(c | (0x80 if n else 0))
        if not n:
            return bytes(out)


def encode_response(pods: list[dict]) -> bytes:
    """Inverse of :func:`decode` (test fixtures and the local kubelet's
    simulated socket)."""
    out = bytearray()
    for p in pods:
        pb = _encode_str(1, p["name"]) + _encode_str(2, p["namespace"])
        for c in p.get("containers", []):
            cb = _encode_str(1, c["name"])
            for d in c.get("devices", []):
                db = _encode_str(1, d["resource_name"]) + b"".join(_encode_str(2, x) for x in d["device_ids"])
                cb += bytes([2 << 3 | 2]) + _enc_varint(len(db)) + db
            pb += bytes([3 << 3 | 2]) + _enc_varint(len(cb)) + cb
        out += bytes([1 << 3 | 2]) + _enc_varint(len(pb)) + pb
    return bytes(out)


# ---------------------------------------------------------------- lookup
def list_pod_resources(socket: str = SOCKET, timeout: float = 5.0) -> list[dict]:
    import grpc

    with grpc.insecure_channel("unix://" + socket) as ch:
        call = ch.unary_unary(LIST_METHOD, request_serializer=lambda _: b"", response_deserializer=lambda b: b)
        return decode(call(None, timeout=timeout))


def allocated_ids(pods: list[dict], name: str, namespace: str, resource: str = "amd.com/gpu",
                  container: str | None = None) -> list[str]:
    for p in pods:
        if p["name"] == name and p["namespace"] == namespace:
            ids = []
            for c in p["containers"]:
                if container and c["name"] != container:
                    continue
                for d in c["devices"]:
                    if d["resource_name"] == resource:
                        ids += d["device_ids"]
            return ids
    raise LookupError(f"pod {namespace}/{name} not in the kubelet's pod-resources list")


_BDF = re.compile(r"^(?:([0-9a-fA-F]{4,8}):)?([0-9a-fA-F]{2}):([0-9a-fA-F]{2})\.([0-7])$")


def parse_bdf(s: str) -> tuple[int, int, int]:
    """'0000:c1:00.0' / 'c1:00.0' -> (domain, bus, device)."""
    m = _BDF.match(s.strip())
    if not m:
        raise ValueError(f"device id {s!r} is not a PCI address")
    return int(m.group(1) or "0", 16), int(m.group(2), 16), int(m.group(3), 16)


def ordinal_for(bdf: tuple[int, int, int], props: list[tuple[int, int, int]]) -> int:
    """HIP ordinal whose (pci_domain_id, pci_bus_id, pci_device_id) is bdf."""
    hits = [i for i, p in enumerate(props) if tuple(p) == tuple(bdf)]
    if len(hits) != 1:
        raise LookupError(f"PCI device {bdf} matches {len(hits)} visible GPUs")
    return hits[0]


def visible_pci() -> list[tuple[int, int, int]]:
    import torch

    out = []
    for i in range(torch.cuda.device_count()):
        p = torch.cuda.get_device_properties(i)
        out.append((int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id)))
    return out


def allocated_device_index(env=os.environ, lister=list_pod_resources, pci=visible_pci) -> int:
    """HIP ordinal of the GPU the kubelet allocated to this pod."""
    name, ns = env.get("TOA_POD_NAME"), env.get("TOA_POD_NAMESPACE")
    if not name or not ns:
        raise RuntimeError("node-local replica without TOA_POD_NAME / TOA_POD_NAMESPACE (downward API)")
    ids = allocated_ids(lister(), name, ns, env.get("TOA_GPU_RESOURCE", "amd.com/gpu"))
    if len(ids) != 1:
        raise RuntimeError(f"pod {ns}/{name} holds {len(ids)} GPUs ({ids}); the node-local layout needs exactly 1")
    return ordinal_for(parse_bdf(ids[0]), pci())
