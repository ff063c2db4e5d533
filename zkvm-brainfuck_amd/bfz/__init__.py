"""bfz — MI355X-native core-proof prover for the felicityin/zkvm-brainfuck zkVM.

The product is libbfz.so (HIP kernels for gfx950 + host C++, C ABI in include/bfz.h);
this package is the host-side mirror of the reference's SDK (crates/sdk) over that ABI.
"""
from ._lib import BfzError, LIB_PATH, init
from .sdk import (BfProofWithPublicValues, BfProvingKey, BfVerifyingKey, Execute, Prove,
                  ProverClient, proof_from_bincode, proof_to_bincode, set_num_queries,
                  set_pcs_variant)
from . import guests

__all__ = ["ProverClient", "BfProvingKey", "BfVerifyingKey", "BfProofWithPublicValues",
           "Execute", "Prove", "BfzError", "LIB_PATH", "init", "set_num_queries", "set_pcs_variant", "proof_to_bincode",
           "proof_from_bincode", "guests"]
