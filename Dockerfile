# Otedama for MI355X: ROCm + PyTorch runtime image.
# Build stage compiles the gfx950 kernels and C++ runtime in-tree; the final
# stage carries only the package, the built extension and its Python deps.
# Run with the GPU device nodes passed through:
#   docker run --device=/dev/kfd --device=/dev/dri --group-add video \
#     -e HSA_ENABLE_IPC_MODE_LEGACY=0 otedama-mi355x run --bitcoin-address bc1q...
ARG BASE=rocm/pytorch:latest

FROM ${BASE} AS builder
WORKDIR /src
COPY csrc csrc
COPY otedama_amd otedama_amd
COPY pyproject.toml README.md ./
RUN python3 -m otedama_amd._build -j 16 && python3 -m compileall -q otedama_amd

FROM ${BASE}
ARG VERSION=dev
ENV OTEDAMA_VERSION=${VERSION} \
    HSA_ENABLE_IPC_MODE_LEGACY=0 \
    PYTHONUNBUFFERED=1
WORKDIR /opt/otedama
COPY --from=builder /src/otedama_amd otedama_amd
COPY config.yaml.example bench.py ./
RUN useradd --system --create-home --groups video,render otedama || true
USER otedama
EXPOSE 3333 3336 9090
ENTRYPOINT ["python3", "-m", "otedama_amd"]
CMD ["run", "--no-tui"]
