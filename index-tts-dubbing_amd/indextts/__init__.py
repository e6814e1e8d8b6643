"""indextts (MI355X-native): drop-in ``indextts.infer.IndexTTS`` whose GPT decode and BigVGAN2 vocoder
run as hand-written HIP kernels (gfx950) behind the C ABI in ``libitts_hip.so``."""
__version__ = "0.1.0"
