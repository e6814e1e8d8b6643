"""torch.profiler view of the C3 prompt-feature phase (conditioning encoder + perceiver + ECAPA) for
32 prompts of 511 frames: device time per op, top entries."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd")]
import torch
from bench import make_inputs
from indextts.pipeline import BatchedTTS
from indextts.utils.config import default_config_path, load_config
from indextts.utils.synthetic import bigvgan_state_dict, gpt_state_dict

cfg = load_config(default_config_path())
dev = torch.device("cuda:0")
tts = BatchedTTS(gpt_state_dict(cfg.gpt, seed=0, mel_head_std=0.08), bigvgan_state_dict(cfg.bigvgan, seed=0),
                 cfg, dev, "bf16", max_kv=600)
tts.graph_features = False  # per-op view (the product replays the same ops as one captured graph)
mels, texts = make_inputs(cfg, list(range(32)), 48, 511)
mels = [m.to(dev) for m in mels]
for _ in range(3):
    tts.prompt_features(mels, None)
torch.cuda.synchronize()
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]) as prof:
    tts.prompt_features(mels, None)
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=30, max_name_column_width=70))
print(prof.key_averages(group_by_stack_n=0).table(sort_by="self_cuda_time_total", row_limit=25, max_name_column_width=60))
