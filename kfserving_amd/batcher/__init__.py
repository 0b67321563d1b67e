"""pkg/batcher semantics: Batcher (core), ModelBatcher (in-process), Agent (HTTP sidecar)."""
from .batcher import Batcher, ModelBatcher, MAX_BATCH_SIZE, MAX_LATENCY_MS  # noqa: F401
