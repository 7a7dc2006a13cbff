"""src/losses/vgg16.py — VGGLoss (VGG16 perceptual loss) on the HIP path (see hyres_hip.vgg)."""
from hyres_hip.vgg import VGGLoss  # noqa: F401
