"""MI355X-native encode -> quantize -> synthesize path of yubster4525/image_compression_2.

Drop-in classes (same names / signatures as the reference modules):
  stylegan3_hvae_full:        HVAE_VGG_Encoder, VGGBlock, HierarchyProjector, StyleGAN3Compressor,
                              save_tensor_as_image
  gumbel_softmax_compression: GumbelSoftmaxDiscretization, GumbelSoftmaxCompressor
  networks_stylegan3:         Generator (G_ema duck type), SynthesisNetwork, SynthesisLayer, ...
  sg3_ops:                    bias_act, upfirdn2d, filtered_lrelu  (torch_utils.ops mirrors)
  cabac_compression:          ContextModel, cabac_encode / cabac_decode, CABACCompressor (native range coder)
  legacy:                     load_network_pkl (SG3 pickle loader that executes nothing from the file)
All compute runs in libic2ops.so (hand-written HIP for gfx950); ROCm tensors only.
"""
from . import _native  # noqa: F401
from .stylegan3_hvae_full import (HVAE_VGG_Encoder, VGGBlock, HierarchyProjector, StyleGAN3Compressor,  # noqa: F401
                                  save_tensor_as_image, quantize_uniform, resize_bilinear)
from .gumbel_softmax_compression import GumbelSoftmaxDiscretization, GumbelSoftmaxCompressor  # noqa: F401
from .networks_stylegan3 import (Generator, SynthesisNetwork, SynthesisLayer, SynthesisInput,  # noqa: F401
                                 MappingNetwork, FullyConnectedLayer, make_generator)
from . import sg3_ops  # noqa: F401
from .cabac_compression import CABACCompressor, ContextModel, cabac_encode, cabac_decode  # noqa: F401
from . import legacy  # noqa: F401

__all__ = ["HVAE_VGG_Encoder", "VGGBlock", "HierarchyProjector", "StyleGAN3Compressor", "save_tensor_as_image",
           "GumbelSoftmaxDiscretization", "GumbelSoftmaxCompressor", "Generator", "SynthesisNetwork",
           "SynthesisLayer", "SynthesisInput", "MappingNetwork", "FullyConnectedLayer", "make_generator",
           "quantize_uniform", "resize_bilinear", "sg3_ops", "CABACCompressor", "ContextModel", "cabac_encode",
           "cabac_decode", "legacy"]
