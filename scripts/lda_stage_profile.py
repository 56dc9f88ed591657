#!/usr/bin/env python
"""Where the pipeline's `lda` stage spends its time beyond the EM iterations (verdict r2 item 5).

Runs ``estimate`` (the stage's body: engine setup, EM with the 000 / final saves, model copies, the
final word-assignment pass) on the synthetic headline day twice -- the first run loads the code
objects -- and prints the stage timing of the second plus its top functions under cProfile.

  python scripts/lda_stage_profile.py [--events 1000000] [--topics 20] [--out gpurun_out/lda_stage.txt]
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=1_000_000)
    ap.add_argument("--topics", type=int, default=20)
    ap.add_argument("--top", type=int, default=35)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from oni_ml_amd.models.lda.estimate import estimate
    from oni_ml_amd.models.lda.settings import LDASettings
    from oni_ml_amd.pipeline.flow import synthetic_flow_corpus

    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    corpus, _ = synthetic_flow_corpus(events=a.events, seed=0, device=dev)
    lines = [f"corpus: {corpus.num_docs} docs, {corpus.num_terms} words, {corpus.nnz} entries; K = {a.topics}"]
    for rep in range(2):
        tmp = tempfile.mkdtemp(prefix="oni_lda_stage_")
        try:
            prof = cProfile.Profile() if rep == 1 else None
            if dev.type == "cuda":
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            if prof:
                prof.enable()
            res = estimate(corpus, a.topics, 2.5, LDASettings(), "random", tmp, backend="auto", device=dev,
                           write_word_assignments=True, defer_files=True)
            if dev.type == "cuda":
                torch.cuda.synchronize()
            t1 = time.perf_counter()
            res.close_files()
            t2 = time.perf_counter()
            if prof:
                prof.disable()
            lines.append(f"run {rep}: estimate {t1 - t0:.4f} s (+ deferred file close {t2 - t1:.4f} s), "
                         f"{res.em_iterations} EM iterations, timing {json.dumps(res.timing)}")
            if prof:
                s = io.StringIO()
                pstats.Stats(prof, stream=s).sort_stats("cumulative").print_stats(a.top)
                lines.append(s.getvalue())
                s = io.StringIO()
                pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(a.top)
                lines.append(s.getvalue())
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
    text = "\n".join(lines)
    print(text, flush=True)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
