//! `HipProver`: the reference's `MachineProver` trait (crates/stark/src/prover.rs:27-150)
//! implemented over libbfz, the MI355X core prover.  Every method maps to one C ABI call:
//!
//! | trait method (reference)                     | libbfz                                   |
//! |----------------------------------------------|------------------------------------------|
//! | `setup` (prover.rs:49, machine.rs:154-224)   | `bfz_setup` (cached per program)          |
//! | `commit` (prover.rs:209-236)                 | `bfz_main_commit` -> `bfz_main_data`      |
//! | `observe_into` (prover.rs:595-601)           | native Rust (same as StarkProvingKey)     |
//! | `open` (prover.rs:242-553)                   | `bfz_open` + `bfz_proof_to_bincode`       |
//! | `prove` (prover.rs:560-582)                  | generate_dependencies + commit + open     |
//!
//! The proof comes back as the reference's own bincode `ShardProof<KoalaBearPoseidon2>` bytes
//! (bfz_proof_to_bincode, `FIELD_MONTGOMERY`), so `bincode::deserialize` yields the exact type
//! `StarkMachine::verify` takes: no hand-written decoder on the Rust side.
//!
//! Not compiled here: the binding mirrors `zkvm-brainfuck_amd/bfz/sdk.py`
//! (`CoreProver.commit / observe_into / open / prove`), which the GPU tests exercise.
use std::ffi::CString;
use std::os::raw::c_int;

use bf_core_executor::{ExecutionRecord, Opcode, Program};
use bf_core_machine::brainfuck::BfAir;
use bf_prover::components::BfProverComponents;
use bf_stark::koala_bear_poseidon2::KoalaBearPoseidon2;
use bf_stark::{
    Challenger, Com, DebugConstraintBuilder, MachineProof, MachineProver, MachineProvingKey,
    MachineRecord, ShardMainData, ShardProof, StarkGenericConfig, StarkMachine, StarkProvingKey,
    StarkVerifyingKey,
};
use bfz_sys as sys;
use p3_challenger::CanObserve;
use p3_field::{FieldAlgebra, PrimeField32};
use p3_koala_bear::KoalaBear;
use p3_matrix::{dense::RowMajorMatrix, Matrix};

type SC = KoalaBearPoseidon2;
type Air = BfAir<KoalaBear>;

/// BfAir::chips() order (crates/core/machine/src/brainfuck/mod.rs:53-81) = chip id in the ABI.
pub const CHIPS: [&str; 8] =
    ["Cpu", "Program", "AddSub", "Jump", "Memory", "Byte", "MemoryInstrs", "IO"];
/// bfz_proof_to_bincode field representation: raw Montgomery word (MontyField31 serde).
pub const FIELD_MONTGOMERY: c_int = 0;

fn chip_id(name: &str) -> c_int {
    CHIPS.iter().position(|c| *c == name).unwrap_or_else(|| panic!("unknown chip {name}")) as c_int
}

/// Program::from (crates/core/executor/src/program.rs:22-45) inverted: the text bfz_setup takes.
pub fn program_source(p: &Program) -> String {
    p.instructions
        .iter()
        .map(|i| match i.opcode {
            Opcode::LoopStart => '[',
            Opcode::LoopEnd => ']',
            Opcode::Add => '+',
            Opcode::Sub => '-',
            Opcode::MemStepForward => '>',
            Opcode::MemStepBackward => '<',
            Opcode::Input => ',',
            Opcode::Output => '.',
        })
        .collect()
}

/// `KoalaBear` is `#[repr(transparent)]` over its Montgomery `u32`.
fn words<T>(v: &[T]) -> &[u32] {
    assert_eq!(core::mem::size_of::<T>(), 4);
    unsafe { core::slice::from_raw_parts(v.as_ptr() as *const u32, v.len()) }
}

#[derive(Debug, Clone, Copy)]
pub struct HipProverError;
impl core::fmt::Display for HipProverError {
    fn fmt(&self, f: &mut core::fmt::Formatter<'_>) -> core::fmt::Result {
        write!(f, "HipProverError")
    }
}
impl std::error::Error for HipProverError {}

/// Device proving key: the host key (commit, preprocessed traces) plus the libbfz handle whose
/// LDEs and Merkle tree stay in HBM.
pub struct HipProvingKey {
    pub host: StarkProvingKey<SC>,
    pub dev: *mut sys::bfz_pk,
}
unsafe impl Send for HipProvingKey {}
unsafe impl Sync for HipProvingKey {}
impl Drop for HipProvingKey {
    fn drop(&mut self) {
        unsafe { sys::bfz_pk_free(self.dev) }
    }
}
impl MachineProvingKey<SC> for HipProvingKey {
    fn preprocessed_commit(&self) -> Com<SC> {
        self.host.commit.clone()
    }
    fn observe_into(&self, challenger: &mut Challenger<SC>) {
        // prover.rs:595-601
        challenger.observe(self.host.commit.clone());
        for _ in 0..7 {
            challenger.observe(KoalaBear::ZERO);
        }
    }
}

/// `DeviceProverData`: the main commit's LDEs and tree in HBM (bfz_main_data), freed on drop.
pub struct HipMainData(*mut sys::bfz_main_data);
unsafe impl Send for HipMainData {}
unsafe impl Sync for HipMainData {}
impl Drop for HipMainData {
    fn drop(&mut self) {
        unsafe { sys::bfz_main_data_free(self.0) }
    }
}

pub struct HipProver {
    machine: StarkMachine<SC, Air>,
}

fn to_c(ch: &Challenger<SC>) -> sys::bfz_challenger {
    // p3 DuplexChallenger keeps sponge_state / input_buffer / output_buffer as pub fields
    let mut c = sys::bfz_challenger::default();
    c.sponge_state.copy_from_slice(words(&ch.sponge_state));
    c.input_buffer[..ch.input_buffer.len()].copy_from_slice(words(&ch.input_buffer));
    c.n_input = ch.input_buffer.len() as u32;
    c.output_buffer[..ch.output_buffer.len()].copy_from_slice(words(&ch.output_buffer));
    c.n_output = ch.output_buffer.len() as u32;
    c
}

impl MachineProver<SC, Air> for HipProver {
    type DeviceMatrix = RowMajorMatrix<KoalaBear>;
    type DeviceProverData = HipMainData;
    type DeviceProvingKey = HipProvingKey;
    type Error = HipProverError;

    fn new(machine: StarkMachine<SC, Air>) -> Self {
        let device = std::env::var("BFZ_DEVICE").ok().and_then(|d| d.parse().ok()).unwrap_or(0);
        sys::check(unsafe { sys::bfz_init(device) });
        Self { machine }
    }

    fn machine(&self) -> &StarkMachine<SC, Air> {
        &self.machine
    }

    fn setup(&self, program: &Program) -> (HipProvingKey, StarkVerifyingKey<SC>) {
        let (host, vk) = self.machine.setup(program);
        let src = CString::new(program_source(program)).unwrap();
        let mut dev = core::ptr::null_mut();
        let mut root = [0u32; 8];
        sys::check(unsafe { sys::bfz_setup(src.as_ptr(), &mut dev, root.as_mut_ptr()) });
        // the device and host preprocessed commitments agree (both are MerkleTreeMmcs roots)
        assert_eq!(words(host.commit.as_ref()), &root[..], "preprocessed commit mismatch");
        (HipProvingKey { host, dev }, vk)
    }

    fn pk_to_device(&self, _pk: &StarkProvingKey<SC>) -> HipProvingKey {
        // keys are made by setup(program): libbfz builds the preprocessed LDEs from the program
        unimplemented!("HipProver: create device keys with setup()")
    }

    fn pk_to_host(&self, pk: &HipProvingKey) -> StarkProvingKey<SC> {
        pk.host.clone()
    }

    fn commit(
        &self,
        mut named_traces: Vec<(String, RowMajorMatrix<KoalaBear>)>,
    ) -> ShardMainData<SC, RowMajorMatrix<KoalaBear>, HipMainData> {
        // prover.rs:214: the same order libbfz commits in (it re-sorts identically)
        named_traces.sort_by_key(|(name, t)| (core::cmp::Reverse(t.height()), name.clone()));
        let ids: Vec<c_int> = named_traces.iter().map(|(n, _)| chip_id(n)).collect();
        let ptrs: Vec<*const u32> =
            named_traces.iter().map(|(_, t)| words(&t.values).as_ptr()).collect();
        let hs: Vec<usize> = named_traces.iter().map(|(_, t)| t.height()).collect();
        let ws: Vec<usize> = named_traces.iter().map(|(_, t)| t.width()).collect();
        let mut data = core::ptr::null_mut();
        let mut root = [0u32; 8];
        sys::check(unsafe {
            sys::bfz_main_commit(core::ptr::null(), ids.as_ptr(), ptrs.as_ptr(), hs.as_ptr(),
                                 ws.as_ptr(), ids.len(), &mut data, root.as_mut_ptr())
        });
        let chip_ordering =
            named_traces.iter().enumerate().map(|(i, (name, _))| (name.to_owned(), i)).collect();
        let main_commit: Com<SC> = unsafe { core::mem::transmute_copy(&root) };
        let traces = named_traces.into_iter().map(|(_, t)| t).collect();
        ShardMainData::new(traces, main_commit, HipMainData(data), chip_ordering)
    }

    fn open(
        &self,
        pk: &HipProvingKey,
        data: ShardMainData<SC, RowMajorMatrix<KoalaBear>, HipMainData>,
        challenger: &mut Challenger<SC>,
    ) -> Result<ShardProof<SC>, HipProverError> {
        let ch = to_c(challenger);
        let (mut p, mut len) = (core::ptr::null_mut(), 0usize);
        sys::check(unsafe { sys::bfz_open(pk.dev, data.main_data.0, &ch, &mut p, &mut len) });
        let bfz1 = unsafe { sys::take_bytes(p, len) };
        let (mut b, mut blen) = (core::ptr::null_mut(), 0usize);
        sys::check(unsafe {
            sys::bfz_proof_to_bincode(bfz1.as_ptr(), bfz1.len(), FIELD_MONTGOMERY, &mut b, &mut blen)
        });
        let bytes = unsafe { sys::take_bytes(b, blen) };
        // the reference's own wire format (utils/prove.rs:46): deserialize straight into the type
        bincode::deserialize(&bytes).map_err(|_| HipProverError)
    }

    fn prove(
        &self,
        pk: &HipProvingKey,
        record: &mut ExecutionRecord,
        challenger: &mut Challenger<SC>,
    ) -> Result<MachineProof<SC>, HipProverError>
    where
        Air: for<'a> p3_air::Air<DebugConstraintBuilder<'a, KoalaBear, <SC as StarkGenericConfig>::Challenge>>,
    {
        self.machine().generate_dependencies(record, None); // prover.rs:570
        pk.observe_into(challenger);
        let traces = self.generate_traces(record);
        let data = self.commit(traces);
        let shard_proof = self.open(pk, data, &mut challenger.clone())?; // prover.rs:578
        Ok(MachineProof { shard_proof })
    }
}

impl HipProver {
    /// Pipelined proofs of one program over many inputs (bfz_prove_batch): execution and event
    /// upload of job k+1 run under the GPU proof of job k.  Returns the reference's bincode
    /// ShardProof bytes per input.
    pub fn prove_batch(&self, pk: &HipProvingKey, stdins: &[Vec<u8>]) -> Vec<ShardProof<SC>> {
        let ptrs: Vec<*const u8> = stdins.iter().map(|s| s.as_ptr()).collect();
        let lens: Vec<usize> = stdins.iter().map(|s| s.len()).collect();
        let mut outs = vec![core::ptr::null_mut(); stdins.len()];
        let mut olens = vec![0usize; stdins.len()];
        sys::check(unsafe {
            sys::bfz_prove_batch(pk.dev, ptrs.as_ptr(), lens.as_ptr(), stdins.len(), 0,
                                 outs.as_mut_ptr(), olens.as_mut_ptr(), core::ptr::null_mut())
        });
        outs.into_iter()
            .zip(olens)
            .map(|(p, n)| {
                let bfz1 = unsafe { sys::take_bytes(p, n) };
                let (mut b, mut blen) = (core::ptr::null_mut(), 0usize);
                sys::check(unsafe {
                    sys::bfz_proof_to_bincode(bfz1.as_ptr(), bfz1.len(), FIELD_MONTGOMERY, &mut b,
                                              &mut blen)
                });
                bincode::deserialize(&unsafe { sys::take_bytes(b, blen) }).expect("bincode")
            })
            .collect()
    }
}

/// crates/prover/src/components.rs:11-20: select the HIP core prover.
pub struct HipProverComponents;
impl BfProverComponents for HipProverComponents {
    type CoreProver = HipProver;
}
