"""MI355X-native (gfx950) Unet3D denoising path of SeanNobel/DALLE2-video.

Drop-in: `from dalle2_video.dalle2_video import Unet3D, VideoDecoder` and
`from dalle2_video.trainer import VideoDecoderTrainer` (train_decoder.py:15-17).
"""
