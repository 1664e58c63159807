"""Prometheus metrics for the extender and the device plugin.

The reference exports none (beego log files + /inspect only).
Here: request counters and latency histograms per verb, apiserver round-trip
latency, bind outcomes, and ledger gauges (per-device used / total gpu-mem,
binpack utilisation) that are computed at scrape time from the native ledger.
"""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest
from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily, HistogramMetricFamily

LAT_BUCKETS = (0.0001, 0.00025, 0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0)


class _LedgerCollector:
    def __init__(self, engine):
        self.engine = engine

    def collect(self):
        used = GaugeMetricFamily("gpushare_device_used_gpu_mem", "gpu-mem accounted on a device",
                                 labels=["node", "device"])
        total = GaugeMetricFamily("gpushare_device_total_gpu_mem", "gpu-mem capacity of a device",
                                  labels=["node", "device"])
        util = GaugeMetricFamily("gpushare_binpack_utilization", "sum(used)/sum(total) over gpushare nodes")
        pods = GaugeMetricFamily("gpushare_ledger_pods", "pods tracked by the ledger")
        unacc = GaugeMetricFamily("gpushare_device_unaccounted_gpu_mem",
                                  "gpu-mem the node's device plugin reports held by containers the annotations put "
                                  "elsewhere (a kubelet swap not yet repaired); charged on top of the annotations",
                                  labels=["node", "device"])
        su = st = 0
        for n in self.engine.node_names():
            for i, (t, u) in enumerate(self.engine.node_devices(n)):
                used.add_metric([n, str(i)], u)
                total.add_metric([n, str(i)], t)
                su += u
                st += t
            if hasattr(self.engine, "node_unaccounted"):
                for i, x in enumerate(self.engine.node_unaccounted(n)):
                    unacc.add_metric([n, str(i)], x)
        util.add_metric([], (su / st) if st else 0.0)
        s = self.engine.stats()
        pods.add_metric([], s["pods"])
        yield used
        yield total
        yield util
        yield pods
        yield unacc
        for k in ("filter_calls", "assume_ok", "assume_fail", "bind_ok", "bind_fail", "expired", "expiry_deferred",
                  "overcommit_events", "pod_upserts", "pod_removes", "moves_ok", "moves_refused",
                  "partner_claims_refused", "unaccounted_updates", "unaccounted_expired"):
            if k not in s:
                continue
            g = GaugeMetricFamily(f"gpushare_engine_{k}", f"native engine counter {k}")
            g.add_metric([], s[k])
            yield g
        if "bind_order_waits" in s:
            c = CounterMetricFamily("gpushare_bind_order_waits", "binds held back to keep a node's equal-size "
                                    "bindings in ASSUME_TIME order")
            c.add_metric([], s["bind_order_waits"])
            yield c
            c = CounterMetricFamily("gpushare_bind_order_wait_seconds", "time binds spent held back for ASSUME_TIME "
                                    "order")
            c.add_metric([], s["bind_order_wait_s"])
            yield c
        # C++ front end (native/engine/server.cc): request counters + latency histograms
        ns = self.engine.server_stats() if hasattr(self.engine, "server_stats") else {}
        if ns:
            for k in ("requests", "filters", "binds", "bind_ok", "bind_fail", "proxied", "bad_requests", "inspects",
                      "connections", "api_calls", "conflicts_retried"):
                c = CounterMetricFamily(f"gpushare_native_{k}", f"native HTTP front end: {k}")
                c.add_metric([], ns[k])
                yield c
            for k in ("filter_latency", "bind_latency", "api_latency"):
                h = ns[k]
                cum, buckets = 0, []
                for le, cnt in zip(h["bounds"], h["counts"]):
                    cum += cnt
                    buckets.append((repr(le), cum))
                buckets.append(("+Inf", cum + h["counts"][-1]))
                yield HistogramMetricFamily(f"gpushare_native_{k}_seconds", f"native {k.replace('_', ' ')}",
                                            buckets=buckets, sum_value=h["sum"])


class Metrics:
    def __init__(self, engine=None, prefix: str = "gpushare"):
        self.registry = CollectorRegistry(auto_describe=True)
        self.requests = Counter(f"{prefix}_http_requests", "extender HTTP requests", ["verb", "code"],
                                registry=self.registry)
        self.latency = Histogram(f"{prefix}_verb_latency_seconds", "extender verb latency", ["verb"],
                                 buckets=LAT_BUCKETS, registry=self.registry)
        self.api_latency = Histogram(f"{prefix}_apiserver_latency_seconds", "apiserver round-trip latency",
                                     ["call"], buckets=LAT_BUCKETS, registry=self.registry)
        self.bind_results = Counter(f"{prefix}_bind_results", "bind outcomes", ["result"], registry=self.registry)
        self.allocate_results = Counter(f"{prefix}_allocate_results", "device-plugin Allocate outcomes",
                                        ["result"], registry=self.registry)
        self.annotation_repairs = Counter(f"{prefix}_bind_annotation_repairs",
                                          "pods bound without the annotations their Binding carried, written back",
                                          ["result"], registry=self.registry)
        self.bind_mode = Gauge(f"{prefix}_bind_mode_update", "1: binds annotate then bind (reference's two calls)",
                               registry=self.registry)
        if engine is not None:
            self.registry.register(_LedgerCollector(engine))

    def render(self) -> bytes:
        return generate_latest(self.registry)
