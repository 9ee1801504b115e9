"""tritonk8ssupervisor_amd — MI355X-native cluster bring-up (control plane + GPU workers).

Same capabilities and public surface as cheapRoc/tritonK8ssupervisor (``./setup.sh`` wizard,
``./setup.sh -c`` teardown, ``terraform/{master,host}`` + ``ansible/clusterUp.yml`` layout), but
targeting one 8x AMD Instinct MI355X (gfx950) node: a local provider instead of Joyent Triton,
an in-repo control plane + node agents instead of Rancher 1.x, and a native HIP/RCCL validation
stack (device discovery, HBM/MD5/xGMI probes, RCCL all-reduce) that must pass before a GPU
worker counts as Ready. See SURVEY.md for the reference map.

Keep this module import-light: node agents and the control plane start as separate processes
and their start-up time is part of the bring-up metric.
"""

__version__ = "0.1.0"
