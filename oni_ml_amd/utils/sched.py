"""CPU priority of the background writer threads.

The config-5 pipeline formats ~49 GB of text (the reference's file contract) on writer threads while
the later stages run; each writer's native formatter starts a thread per core.  Left at the stages'
priority, those threads (two lda model writers + the lda_pre and lda_post writers, 16 format threads
each) crowd out the thread that drives the GPU: the 25 EM iterations of config 5 measured 5.9 s on
an idle host and 9.3 s beside the writers.  A writer thread raises its own nice value when it starts;
the native threads it creates inherit it, so the formatting fills the cycles the stages leave idle.
"""
import os
import threading


BG_NICE = 10     # background writers' nice value: they take the cycles the stages leave

def background_priority() -> None:
    """Raise the calling thread's nice value by BG_NICE (10).  Linux
    applies PRIO_PROCESS with a thread id to that thread only; raising a nice value needs no
    privilege.  Best effort: other platforms or a refused call leave the priority as it is."""
    n = BG_NICE
    if n <= 0 or not hasattr(os, "setpriority"):
        return
    try:
        tid = threading.get_native_id()
        cur = os.getpriority(os.PRIO_PROCESS, tid)
        os.setpriority(os.PRIO_PROCESS, tid, min(19, cur + n))
    except OSError:
        pass
