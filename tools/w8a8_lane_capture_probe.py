"""Round 6 diagnostic: capture the W8A8 row-lane forward (vit_b, B = 1) into a HIP graph, replay it and
compare with one chain (run it in its own process: a capture failure ends only that process).
Measured on MI355X: with pairwise cross-stream events for the global blocks (lane i waiting on an
event recorded on lane j) the capture crashed in capture_end (SIGSEGV, eager forward bit-identical);
joins through the forking stream (the form kept in W8A8Engine._blocks_row_lanes) capture and replay
bit-identically (profiles/r6_w8a8_row_lanes.log)."""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "sam-quantization_amd"))
from samq.synthetic import random_fq_encoder  # noqa: E402

dev = torch.device("cuda:0")
enc = random_fq_encoder("vit_b", device=dev)
eng = enc.engine()
img = torch.randn((1, 3, 1024, 1024), generator=torch.Generator(device=dev).manual_seed(5), device=dev)
eng.row_lanes = 1
ref = eng(img).clone()
eng.row_lanes = 2
print("eager identical:", torch.equal(eng(img), ref), flush=True)
graph, out = eng.capture(img)
print("captured", flush=True)
graph.replay()
torch.cuda.synchronize()
print("graph identical:", torch.equal(out, ref), flush=True)
