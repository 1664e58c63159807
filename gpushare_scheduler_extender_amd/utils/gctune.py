"""Garbage-collector settings for the long-running control-plane processes.

The informer stores hold tens of thousands of small dicts; CPython's default
generation-0 threshold (700 allocations) makes the cyclic collector walk them
every few hundred events, and a full collection stalls the event loop for
milliseconds in the middle of a scheduling wave.  Everything allocated during
start-up is moved to the permanent generation (``gc.freeze``) and the young
generation threshold is raised; pods and events are acyclic JSON trees, so
reference counting frees them without the cyclic collector.
"""
import gc


def tune(gen0: int = 50_000, gen1: int = 50, gen2: int = 100) -> None:
    gc.collect()
    gc.freeze()
    gc.set_threshold(gen0, gen1, gen2)
