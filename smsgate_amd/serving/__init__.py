"""GPU serving runtime of the local extractor: schema FSM, engine, worker thread."""
from .fsm import DEFAULT_FIELDS, FieldSpec, SchemaFSM, build_fsm  # noqa: F401


def freeze_gc_for_launch_loop() -> None:
    """GC policy for a process that launches GPU work from Python (engine server,
    bench rank): freeze the long-lived objects created during init and make
    full (gen-2) collections rare.  A gen-2 pass over the engine's objects stalls
    the kernel-launch stream for milliseconds; measured +5 % msgs/s at the
    headline config (profiles/r01b_gc_ab.txt)."""
    import gc

    gc.collect()
    gc.freeze()
    gc.set_threshold(50_000, 50, 1000)
