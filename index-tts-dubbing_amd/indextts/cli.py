"""``indextts`` command line (reference ``indextts/cli.py:7-59``): same arguments and checks; the
device defaults to the first HIP GPU and there is no CPU mode."""
from __future__ import annotations

import argparse
import os
import sys


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="IndexTTS Command Line")
    p.add_argument("text", type=str, help="Text to be synthesized")
    p.add_argument("-v", "--voice", type=str, required=True, help="Path to the audio prompt file (wav format)")
    p.add_argument("-o", "--output_path", type=str, default="gen.wav", help="Path to the output wav file")
    p.add_argument("-c", "--config", type=str, default="checkpoints/config.yaml",
                   help="Path to the config file. Default is 'checkpoints/config.yaml'")
    p.add_argument("--model_dir", type=str, default="checkpoints",
                   help="Path to the model directory. Default is 'checkpoints'")
    p.add_argument("--fp16", action="store_true", default=True, help="Use FP16 for inference if available")
    p.add_argument("-f", "--force", action="store_true", default=False,
                   help="Force to overwrite the output file if it exists")
    p.add_argument("-d", "--device", type=str, default=None, help="Device to run the model on (cuda, cuda:N).")
    return p


def main(argv=None) -> int:
    parser = build_parser()
    args = parser.parse_args(argv)
    problems = [
        (len(args.text.strip()) == 0, "ERROR: Text is empty."),
        (not os.path.exists(args.voice), f"Audio prompt file {args.voice} does not exist."),
        (not os.path.exists(args.config), f"Config file {args.config} does not exist."),
    ]
    for bad, msg in problems:
        if bad:
            print(msg)
            parser.print_help()
            return 1
    if os.path.exists(args.output_path):
        if not args.force:
            print(f"ERROR: Output file {args.output_path} already exists. Use --force to overwrite.")
            parser.print_help()
            return 1
        os.remove(args.output_path)
    import torch
    if args.device is None:
        if not torch.cuda.is_available():
            print("ERROR: no ROCm GPU visible; this build has no CPU mode.")
            return 1
        args.device = "cuda:0"
    from indextts.infer import IndexTTS
    tts = IndexTTS(cfg_path=args.config, model_dir=args.model_dir, is_fp16=args.fp16, device=args.device)
    tts.infer(audio_prompt=args.voice, text=args.text.strip(), output_path=args.output_path)
    return 0


if __name__ == "__main__":
    sys.exit(main())
