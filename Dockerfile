# MI355X (gfx950) image: ROCm 7.x + PyTorch-ROCm, then the in-tree native build.
ARG BASE=rocm/pytorch:latest
FROM ${BASE}
ENV PYTORCH_ROCM_ARCH=gfx950 \
    HSA_ENABLE_IPC_MODE_LEGACY=0
WORKDIR /workspace/ml-recipe
COPY requirements.txt .
RUN pip install --no-cache-dir -r requirements.txt
COPY . .
# hipcc --offload-arch=gfx950 kernels + g++ host runtime, in-tree
RUN python -m ml_recipe_distributed_pytorch_amd.csrc.build -j 16 && python -c "import __graft_entry__ as g; g.build()"
CMD ["bash", "scripts/run_distributed_on_single_node.sh", "-c", "config/test_bert.cfg"]
