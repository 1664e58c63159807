"""kube-scheduler extender wire types.

The reference (de)serialises the *internal* scheduler API structs, which
carry no ``json:`` tags (``vendor/k8s.io/kubernetes/pkg/scheduler/api/types.go:258-302``):
responses use the Go field names verbatim (``NodeNames``, ``FailedNodes``,
``Error``) and requests are matched case-insensitively by Go's decoder, so both
the legacy (``Pod``/``NodeNames``) and the modern v1 (``pod``/``nodenames``)
kube-scheduler spellings work.  These helpers reproduce exactly that.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field


def ci_get(d: dict, key: str, default=None):
    """Go encoding/json field matching: exact key first, else ASCII case-insensitive (last wins)."""
    if key in d:
        return d[key]
    kl = key.lower()
    hit = default
    for k, v in d.items():
        if isinstance(k, str) and k.lower() == kl:
            hit = v
    return hit


class WireError(ValueError):
    pass


@dataclass
class ExtenderBindingArgs:
    """types.go:287-296."""

    pod_name: str
    pod_namespace: str
    pod_uid: str
    node: str

    @classmethod
    def decode(cls, body: bytes) -> "ExtenderBindingArgs":
        try:
            d = json.loads(body)
        except (ValueError, UnicodeDecodeError) as e:
            raise WireError(str(e)) from e
        if not isinstance(d, dict):
            raise WireError("json: cannot unmarshal value into Go value of type api.ExtenderBindingArgs")

        def s(k):
            v = ci_get(d, k, "")
            if v is None:
                return ""
            if not isinstance(v, str):
                raise WireError(f"json: cannot unmarshal {type(v).__name__} into Go struct field "
                                f"ExtenderBindingArgs.{k} of type string")
            return v

        return cls(s("PodName"), s("PodNamespace"), s("PodUID"), s("Node"))

    def encode(self) -> bytes:
        return json.dumps({"PodName": self.pod_name, "PodNamespace": self.pod_namespace,
                           "PodUID": self.pod_uid, "Node": self.node}, separators=(",", ":")).encode()


def binding_result(error: str = "") -> bytes:
    """types.go:299-302 -> {"Error":""}."""
    return json.dumps({"Error": error}, separators=(",", ":")).encode()


def watch_object_bytes(line: bytes | None) -> bytes | None:
    """The ``object`` of a watch event line ``{"type":"...","object":{...}}``, without re-encoding.

    Returns None unless the line has exactly that shape (what kube-apiserver and
    the fake apiserver emit); callers fall back to ``json.dumps``.
    """
    if not line or not line.startswith(b'{"type":"'):
        return None
    i = line.find(b'","object":', 9)
    if i < 0:
        return None
    end = len(line.rstrip())
    if end < 1 or line[end - 1:end] != b"}":
        return None
    obj = line[i + 11:end - 1]
    return obj if obj[:1] == b"{" and obj[-1:] == b"}" else None


def filter_args_raw(pod_json: bytes, node_names: list[str]) -> bytes:
    """:func:`filter_args` for a pod already serialised (NodeNames form)."""
    names = json.dumps(node_names, separators=(",", ":")).encode()
    return b'{"Pod":' + pod_json + b',"Nodes":null,"NodeNames":' + names + b"}"


def filter_args(pod: dict, node_names: list[str] | None = None, nodes: list[dict] | None = None) -> bytes:
    """ExtenderArgs as kube-scheduler sends it (nodeCacheCapable -> NodeNames)."""
    d = {"Pod": pod, "Nodes": None, "NodeNames": node_names}
    if nodes is not None:
        d["Nodes"] = {"metadata": {}, "items": nodes}
        d["NodeNames"] = None
    return json.dumps(d, separators=(",", ":")).encode()


@dataclass
class ExtenderFilterResult:
    node_names: list[str] | None
    failed_nodes: dict[str, str] = field(default_factory=dict)
    error: str = ""
    nodes: dict | None = None

    @classmethod
    def decode(cls, body: bytes) -> "ExtenderFilterResult":
        d = json.loads(body)
        return cls(ci_get(d, "NodeNames"), ci_get(d, "FailedNodes") or {}, ci_get(d, "Error") or "",
                   ci_get(d, "Nodes"))

    def passing(self) -> list[str]:
        if self.node_names is not None:
            return list(self.node_names)
        if self.nodes:
            return [((n.get("metadata") or {}).get("name", "")) for n in self.nodes.get("items") or []]
        return []


# ---------------------------------------------------------------- inspect schema
# pkg/scheduler/gpushare-inspect.go:14-38 (lowercase json tags)

@dataclass
class InspectPod:
    name: str
    namespace: str
    usedGPU: int


@dataclass
class InspectDevice:
    id: int
    totalGPU: int
    usedGPU: int
    pods: list[InspectPod]


@dataclass
class InspectNode:
    name: str
    totalGPU: int
    usedGPU: int
    devs: list[InspectDevice]


@dataclass
class InspectResult:
    nodes: list[InspectNode]
    error: str = ""

    @classmethod
    def decode(cls, body: bytes | str | dict) -> "InspectResult":
        d = body if isinstance(body, dict) else json.loads(body)
        nodes = []
        for n in d.get("nodes") or []:
            devs = [InspectDevice(x["id"], x["totalGPU"], x["usedGPU"],
                                  [InspectPod(p["name"], p["namespace"], p["usedGPU"]) for p in x.get("pods") or []])
                    for x in n.get("devs") or []]
            nodes.append(InspectNode(n["name"], n["totalGPU"], n["usedGPU"], devs))
        return cls(nodes, d.get("error", ""))
