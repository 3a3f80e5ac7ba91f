"""llm_message_queue_amd -- an MI355X-native LLM request-routing gateway.

Capabilities of ZhangLearning/llm-message-queue (REST API, 4-level priority
queue, delayed/dead-letter queues, workers with backoff, content
preprocessor, load balancer, endpoint autoscaler, resource scheduler,
conversation state + persistence), re-designed around one MI355X node:

  * native C++ queue core (``_lib/_mlq``) with per-level locks;
  * hand-written CDNA4 HIP kernels (``_lib/_hipops``) for the preprocess
    pipeline (tokenize/hash, keyword scoring, sentiment/question, MFMA
    embedding classifier) and context summarisation, plus the backend
    stub's decode kernels;
  * GPU backends (one process per GPU) coordinated per tick through a
    node-local shared-memory control plane, KV migration over RCCL / xGMI
    (``parallel/``), load signals from amd-smi + device-resident
    in-flight counters (``backend/``).
"""
__version__ = "0.1.0"
