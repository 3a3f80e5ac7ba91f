"""Packaging.  The native extensions (HIP kernels for gfx950, the C++ queue /
ring / ingress / telemetry modules) are compiled in-tree first:

    python -m llm_message_queue_amd._build
    python -m pip wheel . --no-deps --no-build-isolation

and shipped as package data; ``llmq`` is the command-line entry point
(``llmq serve``, ``llmq api-gateway``, ``llmq queue-manager``, ``llmq scheduler``,
``llmq validate-config``, ``llmq token``).
"""
from setuptools import find_packages, setup
from setuptools.dist import Distribution


class _Binary(Distribution):
    """The wheel carries compiled .so files: tag it for the platform."""

    def has_ext_modules(self):
        return True


setup(
    name="llm-message-queue-amd",
    version="1.0.0",
    description="MI355X-native LLM request-routing gateway: 4-tier priority queue, GPU preprocessing, GPU backends",
    long_description=open("README.md", encoding="utf-8").read(),
    long_description_content_type="text/markdown",
    python_requires=">=3.10",
    packages=find_packages(include=["llm_message_queue_amd", "llm_message_queue_amd.*"]),
    package_data={"llm_message_queue_amd": ["_lib/*.so"]},
    install_requires=["torch", "numpy", "fastapi", "uvicorn", "pyyaml", "prometheus_client", "grpcio", "protobuf"],
    extras_require={"test": ["pytest", "pytest-timeout", "hypothesis", "httpx", "aiohttp"]},
    entry_points={"console_scripts": ["llmq = llm_message_queue_amd.cli.main:main"]},
    distclass=_Binary,
)
