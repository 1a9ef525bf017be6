"""FedKSeed (zeroth-order federated fine-tuning with K seeds) on MI355X.

Same module layout and API as the reference's python/fate_llm/algo/fedkseed/; the
seed -> perturbation expansion and the scalar-weighted updates run in libfks.so
(gfx950 HIP kernels, C ABI in include/fks.h) through ``codec``.
"""
