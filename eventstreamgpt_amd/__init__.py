"""eventstreamgpt_amd — an MI355X-native (gfx950) implementation of the Event Stream GPT training step.

The package mirrors the reference's import surface for the hot path (``data.types.PytorchBatch``,
``data.data_embedding_layer.DataEmbeddingLayer``, ``transformer.config.StructuredTransformerConfig``, the CI and
NA point-process transformers and generative heads) while routing the compute through hand-written HIP kernels
in ``csrc/`` exposed through the C ABI declared in ``include/esgpt_amd.h``.
"""

__version__ = "0.1.0"
