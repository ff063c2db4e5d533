//! `HipProver`: the reference's `MachineProver` trait (crates/stark/src/prover.rs:27-150)
//! implemented over libbfz, the MI355X core prover.  Every method maps to C ABI calls:
//!
//! | trait method (reference)                        | libbfz                                      |
//! |-------------------------------------------------|---------------------------------------------|
//! | `setup` (prover.rs:49, machine.rs:154-224)      | host `StarkMachine::setup` + `pk_to_device`  |
//! | `pk_to_device` (prover.rs:52,201-203)           | `bfz_pk_from_host` (checked against commit) |
//! | `pk_to_host` (prover.rs:55,205-207)             | the host key kept beside the handle         |
//! | `commit` (prover.rs:209-236)                    | `bfz_main_commit` -> `bfz_main_data`         |
//! | `observe_into` (prover.rs:595-601)              | native Rust (same as StarkProvingKey)       |
//! | `open` (prover.rs:242-553)                      | `bfz_open` + `bfz_proof_to_bincode`          |
//! | `prove` (prover.rs:560-582)                     | `bfz_record_from_events` + record commit + open |
//!
//! `prove` overrides the default: instead of `generate_dependencies` + `generate_traces` on the
//! host and a 1 GB trace upload, the record's event vectors (~50 B per cycle) go to the device,
//! where every chip trace and the byte-lookup multiplicities are generated.
//!
//! The proof comes back as the reference's own bincode `ShardProof<KoalaBearPoseidon2>` bytes
//! (bfz_proof_to_bincode, `FIELD_MONTGOMERY`), so `bincode::deserialize` yields the exact type
//! `StarkMachine::verify` takes: no hand-written decoder on the Rust side.
//!
//! Selection: this crate does not depend on bf-prover (bf-prover depends on it behind its `hip`
//! feature, which points `DefaultProverComponents::CoreProver` here; see
//! crates/reference-patch/ and INTEGRATION.md).
//!
//! Not compiled here (no Rust toolchain in this image): the binding mirrors
//! `zkvm-brainfuck_amd/bfz/sdk.py` (`BfProver`, `CoreProver`), which the GPU tests exercise.
use std::ffi::CString;
use std::os::raw::c_int;

use bf_core_executor::events::MemoryRecordEnum;
use bf_core_executor::{ExecutionRecord, Opcode, Program};
use bf_core_machine::brainfuck::BfAir;
use bf_stark::koala_bear_poseidon2::KoalaBearPoseidon2;
use bf_stark::{
    Challenger, Com, DebugConstraintBuilder, MachineProof, MachineProver, MachineProvingKey,
    ShardMainData, ShardProof, StarkGenericConfig, StarkMachine, StarkProvingKey,
    StarkVerifyingKey,
};
use bfz_sys as sys;
use hashbrown::HashMap;
use p3_air::Air;
use p3_challenger::CanObserve;
use p3_field::FieldAlgebra;
use p3_koala_bear::KoalaBear;
use p3_matrix::{dense::RowMajorMatrix, Matrix};
use p3_maybe_rayon::prelude::*;
use p3_symmetric::Hash;

type SC = KoalaBearPoseidon2;
type A = BfAir<KoalaBear>;

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
fn field_words(w: &[u32]) -> Vec<KoalaBear> {
    assert_eq!(core::mem::size_of::<KoalaBear>(), 4);
    w.iter().map(|&x| unsafe { core::mem::transmute::<u32, KoalaBear>(x) }).collect()
}

/// This configuration's commitment is MerkleTreeMmcs's `Hash<KoalaBear, KoalaBear, 8>`
/// (`p3_symmetric::Hash: From<[W; N]>`), built here from the device root's Montgomery words: a
/// configuration whose commitment were another type fails to compile instead of being
/// transmuted into.
fn commitment(root: &[u32; 8]) -> Com<SC> {
    let w: [KoalaBear; 8] = field_words(root).try_into().expect("8 digest words");
    Hash::<KoalaBear, KoalaBear, 8>::from(w)
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

/// An `ExecutionRecord`'s events resident in HBM (bfz_record), freed on drop.
struct HipRecord(*mut sys::bfz_record);
impl Drop for HipRecord {
    fn drop(&mut self) {
        unsafe { sys::bfz_record_free(self.0) }
    }
}

pub struct HipProver {
    machine: StarkMachine<SC, A>,
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

fn from_c(c: &sys::bfz_challenger, ch: &mut Challenger<SC>) {
    let st = field_words(&c.sponge_state);
    ch.sponge_state.copy_from_slice(&st);
    ch.input_buffer = field_words(&c.input_buffer[..c.n_input as usize]);
    ch.output_buffer = field_words(&c.output_buffer[..c.n_output as usize]);
}

fn access(a: &Option<MemoryRecordEnum>) -> sys::bfz_memory_access {
    match a {
        None => sys::bfz_memory_access::default(),
        Some(MemoryRecordEnum::Read(r)) => sys::bfz_memory_access {
            kind: 1,
            value: r.value,
            prev_value: 0,
            _pad: 0,
            timestamp: r.timestamp,
            prev_timestamp: r.prev_timestamp,
        },
        Some(MemoryRecordEnum::Write(w)) => sys::bfz_memory_access {
            kind: 2,
            value: w.value,
            prev_value: w.prev_value,
            _pad: 0,
            timestamp: w.timestamp,
            prev_timestamp: w.prev_timestamp,
        },
    }
}

/// The record's event vectors (record.rs:15-34) in the bfz_*_event layouts.
#[allow(dead_code)] // the full hand-over (bfz_record_from_events); prove uses CycleArrays
struct EventArrays {
    cpu: Vec<sys::bfz_cpu_event>,
    add: Vec<sys::bfz_alu_event>,
    sub: Vec<sys::bfz_alu_event>,
    jump: Vec<sys::bfz_jump_event>,
    io: Vec<sys::bfz_io_event>,
    memory_instr: Vec<sys::bfz_mem_instr_event>,
    memory: Vec<sys::bfz_memory_event>,
}

#[allow(dead_code)]
impl EventArrays {
    fn new(r: &ExecutionRecord) -> Self {
        let alu = |e: &bf_core_executor::events::AluEvent| sys::bfz_alu_event {
            pc: e.pc,
            opcode: e.opcode as u8,
            next_mv: e.next_mv,
            mv: e.mv,
            _pad: 0,
        };
        Self {
            cpu: r
                .cpu_events
                .par_iter()
                .map(|e| sys::bfz_cpu_event {
                    clk: e.clk,
                    pc: e.pc,
                    next_pc: e.next_pc,
                    mp: e.mp,
                    next_mp: e.next_mp,
                    mv: e.mv,
                    next_mv: e.next_mv,
                    _pad: [0; 2],
                    mv_access: access(&e.mv_access),
                    next_mv_access: access(&e.next_mv_access),
                })
                .collect(),
            add: r.add_events.par_iter().map(alu).collect(),
            sub: r.sub_events.par_iter().map(alu).collect(),
            jump: r
                .jump_events
                .par_iter()
                .map(|e| sys::bfz_jump_event {
                    pc: e.pc,
                    next_pc: e.next_pc,
                    opcode: e.opcode as u8,
                    _pad: [0; 3],
                    dst: e.dst,
                    mv: e.mv,
                    _pad2: [0; 3],
                })
                .collect(),
            io: r
                .io_events
                .iter()
                .map(|e| sys::bfz_io_event {
                    pc: e.pc,
                    opcode: e.opcode as u8,
                    _pad: [0; 3],
                    mp: e.mp,
                    mv: e.mv,
                    _pad2: [0; 3],
                })
                .collect(),
            memory_instr: r
                .memory_instr_events
                .par_iter()
                .map(|e| sys::bfz_mem_instr_event {
                    clk: e.clk,
                    pc: e.pc,
                    opcode: e.opcode as u8,
                    _pad: [0; 3],
                    mp: e.mp,
                    next_mp: e.next_mp,
                })
                .collect(),
            // HashMap-drain order (executor.rs:74); libbfz sorts it into the normal form
            memory: r
                .cpu_memory_access
                .iter()
                .map(|e| sys::bfz_memory_event {
                    addr: e.addr,
                    initial_timestamp: e.initial_mem_access.timestamp,
                    final_timestamp: e.final_mem_access.timestamp,
                    initial_value: e.initial_mem_access.value,
                    final_value: e.final_mem_access.value,
                    _pad: [0; 2],
                })
                .collect(),
        }
    }

    fn as_c(&self) -> sys::bfz_events {
        sys::bfz_events {
            cpu: self.cpu.as_ptr(),
            n_cpu: self.cpu.len(),
            add: self.add.as_ptr(),
            n_add: self.add.len(),
            sub: self.sub.as_ptr(),
            n_sub: self.sub.len(),
            jump: self.jump.as_ptr(),
            n_jump: self.jump.len(),
            io: self.io.as_ptr(),
            n_io: self.io.len(),
            memory_instr: self.memory_instr.as_ptr(),
            n_memory_instr: self.memory_instr.len(),
            memory: self.memory.as_ptr(),
            n_memory: self.memory.len(),
        }
    }
}

/// `n` values of `T` in page-locked host memory (`bfz_host_alloc`): libbfz DMAs a hand-over
/// array straight from it instead of staging it through its own pinned chunks.
struct PinnedVec<T: Copy> {
    ptr: *mut T,
    len: usize,
}

impl<T: Copy> PinnedVec<T> {
    fn new(len: usize) -> Self {
        let mut p = core::ptr::null_mut();
        sys::check(unsafe { sys::bfz_host_alloc(len.max(1) * core::mem::size_of::<T>(), &mut p) });
        Self { ptr: p as *mut T, len }
    }
    fn as_ptr(&self) -> *const T {
        self.ptr
    }
    fn len(&self) -> usize {
        self.len
    }
    /// Every element is written before it is read (the caller fills the whole slice).
    fn as_mut_slice(&mut self) -> &mut [T] {
        unsafe { core::slice::from_raw_parts_mut(self.ptr, self.len) }
    }
}

impl<T: Copy> Drop for PinnedVec<T> {
    fn drop(&mut self) {
        unsafe { sys::bfz_host_free(self.ptr as *mut core::ffi::c_void) };
    }
}

unsafe impl<T: Copy + Send> Send for PinnedVec<T> {}

/// The compact hand-over of `bfz_record_from_cycles`: one 16-byte `bfz_cycle` per CpuEvent
/// plus the memory events.  The device rebuilds the CpuEvents' derived fields and every chip's
/// events (add/jump/memory_instr/io are the cycles' own fields, executor.rs:196-239), so about
/// 16 B per cycle cross PCIe instead of ~64 B.  The cycles are written in parallel straight into
/// page-locked memory, so the upload is one DMA.
struct CycleArrays {
    cycles: PinnedVec<sys::bfz_cycle>,
    memory: Vec<sys::bfz_memory_event>,
}

fn cycle_of(e: &bf_core_executor::events::CpuEvent) -> sys::bfz_cycle {
    let (prev_ts, prev_value) = match e.mv_access {
        None => (0, 0),
        Some(MemoryRecordEnum::Read(a)) => (a.prev_timestamp, 0),
        Some(MemoryRecordEnum::Write(a)) => (a.prev_timestamp, a.prev_value),
    };
    sys::bfz_cycle { pc: e.pc, mp: e.mp, prev_ts, mv: e.mv, prev_value, _pad: [0; 2] }
}

fn memory_events(r: &ExecutionRecord) -> Vec<sys::bfz_memory_event> {
    // HashMap-drain order (executor.rs:74); libbfz sorts it into the normal form
    r.cpu_memory_access
        .iter()
        .map(|e| sys::bfz_memory_event {
            addr: e.addr,
            initial_timestamp: e.initial_mem_access.timestamp,
            final_timestamp: e.final_mem_access.timestamp,
            initial_value: e.initial_mem_access.value,
            final_value: e.final_mem_access.value,
            _pad: [0; 2],
        })
        .collect()
}

/// Cycles per bfz_cycles_push (2 MB): small enough that the DMA of the first chunks starts while
/// the rest are converted, large enough that the per-copy cost stays small
/// (crates/bf-hip-prover/standin/cycle_arrays.cpp times the same loop; scripts/handover_ab.py:
/// 2^17 cycles 29.9-30.0 ms, 2^15 30.0-30.5, 2^13 33.8, one chunk per thread at 2^19 31.2-31.4).
const HANDOVER_CHUNK: usize = 1 << 17;

impl CycleArrays {
    #[allow(dead_code)] // the one-shot hand-over (bfz_record_from_cycles); prove uses hand_over
    fn new(r: &ExecutionRecord) -> Self {
        let mut cycles = PinnedVec::new(r.cpu_events.len());
        cycles
            .as_mut_slice()
            .par_iter_mut()
            .zip(r.cpu_events.par_iter())
            .for_each(|(o, e)| *o = cycle_of(e));
        Self { cycles, memory: memory_events(r) }
    }

    /// The pipelined hand-over: rayon converts record.cpu_events chunk by chunk into page-locked
    /// memory and each chunk is pushed (bfz_cycles_push) as soon as it is written, so its DMA runs
    /// while the next chunks are converted; bfz_cycles_finish validates, expands and returns the
    /// device record (the same record as bfz_record_from_cycles over CycleArrays::new).
    fn hand_over(pk: *const sys::bfz_pk, r: &ExecutionRecord) -> *mut sys::bfz_record {
        let n = r.cpu_events.len();
        let mut cycles = PinnedVec::<sys::bfz_cycle>::new(n);
        let mut up = core::ptr::null_mut();
        sys::check(unsafe { sys::bfz_cycles_begin(pk, n, &mut up) });
        let up_addr = up as usize; // the handle is only passed back to libbfz (thread-safe calls)
        let failed = core::sync::atomic::AtomicI32::new(0);
        cycles
            .as_mut_slice()
            .par_chunks_mut(HANDOVER_CHUNK)
            .zip(r.cpu_events.par_chunks(HANDOVER_CHUNK))
            .enumerate()
            .for_each(|(k, (o, e))| {
                for (oi, ei) in o.iter_mut().zip(e) {
                    *oi = cycle_of(ei);
                }
                let rc = unsafe {
                    sys::bfz_cycles_push(up_addr as *mut sys::bfz_cycle_upload, k * HANDOVER_CHUNK,
                                         o.as_ptr(), o.len())
                };
                if rc != 0 {
                    failed.store(rc, core::sync::atomic::Ordering::Relaxed);
                }
            });
        if failed.load(core::sync::atomic::Ordering::Relaxed) != 0 {
            unsafe { sys::bfz_cycles_abort(up) };
            sys::check(failed.into_inner());
        }
        let memory = memory_events(r);
        let mut rec = core::ptr::null_mut();
        // finish returns after every copy has landed: the pinned chunks may be freed afterwards
        sys::check(unsafe { sys::bfz_cycles_finish(up, memory.as_ptr(), memory.len(), &mut rec) });
        drop(cycles);
        rec
    }
}

impl HipProver {
    /// BFZ1 proof bytes -> the reference's ShardProof (utils/prove.rs:46 wire format).
    fn shard_proof(bfz1: &[u8]) -> Result<ShardProof<SC>, HipProverError> {
        let (mut b, mut blen) = (core::ptr::null_mut(), 0usize);
        sys::check(unsafe {
            sys::bfz_proof_to_bincode(bfz1.as_ptr(), bfz1.len(), FIELD_MONTGOMERY, &mut b, &mut blen)
        });
        let bytes = unsafe { sys::take_bytes(b, blen) };
        bincode::deserialize(&bytes).map_err(|_| HipProverError)
    }
}

impl MachineProver<SC, A> for HipProver {
    type DeviceMatrix = RowMajorMatrix<KoalaBear>;
    type DeviceProverData = HipMainData;
    type DeviceProvingKey = HipProvingKey;
    type Error = HipProverError;

    fn new(machine: StarkMachine<SC, A>) -> Self {
        let device = std::env::var("BFZ_DEVICE").ok().and_then(|d| d.parse().ok()).unwrap_or(0);
        sys::check(unsafe { sys::bfz_init(device) });
        Self { machine }
    }

    fn machine(&self) -> &StarkMachine<SC, A> {
        &self.machine
    }

    fn setup(&self, program: &Program) -> (HipProvingKey, StarkVerifyingKey<SC>) {
        // the host key is what BfProver::setup keeps (pk_to_host, crates/prover/src/lib.rs:51);
        // the device key is made from it exactly as BfProver::prove does (lib.rs:76)
        let (host, vk) = self.machine.setup(program);
        (self.pk_to_device(&host), vk)
    }

    fn pk_to_device(&self, pk: &StarkProvingKey<SC>) -> HipProvingKey {
        // StarkProvingKey::traces in the key's order; chip_ordering maps each name to its index
        let mut chips = vec![-1 as c_int; pk.traces.len()];
        for (name, &i) in pk.chip_ordering.iter() {
            chips[i] = chip_id(name);
        }
        assert!(chips.iter().all(|&c| c >= 0), "pk_to_device: chip_ordering does not cover the traces");
        let ptrs: Vec<*const u32> = pk.traces.iter().map(|t| words(&t.values).as_ptr()).collect();
        let hs: Vec<usize> = pk.traces.iter().map(|t| t.height()).collect();
        let ws: Vec<usize> = pk.traces.iter().map(|t| t.width()).collect();
        let commit = words(pk.commit.as_ref());
        let mut dev = core::ptr::null_mut();
        // libbfz recovers the program from the Program trace, checks both traces against it and
        // the device commitment against pk.commit (a mismatch is an error, not a silent re-key)
        sys::check(unsafe {
            sys::bfz_pk_from_host(chips.as_ptr(), ptrs.as_ptr(), hs.as_ptr(), ws.as_ptr(),
                                  chips.len(), commit.as_ptr(), &mut dev)
        });
        HipProvingKey { host: pk.clone(), dev }
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
        let main_commit = commitment(&root);
        let traces = named_traces.into_iter().map(|(_, t)| t).collect();
        ShardMainData::new(traces, main_commit, HipMainData(data), chip_ordering)
    }

    fn open(
        &self,
        pk: &HipProvingKey,
        data: ShardMainData<SC, RowMajorMatrix<KoalaBear>, HipMainData>,
        challenger: &mut Challenger<SC>,
    ) -> Result<ShardProof<SC>, HipProverError> {
        let mut ch = to_c(challenger);
        let (mut p, mut len) = (core::ptr::null_mut(), 0usize);
        sys::check(unsafe { sys::bfz_open(pk.dev, data.main_data.0, &mut ch, &mut p, &mut len) });
        // bfz_open advances the challenger through the whole opening, as the trait's open does
        from_c(&ch, challenger);
        let bfz1 = unsafe { sys::take_bytes(p, len) };
        Self::shard_proof(&bfz1)
    }

    fn prove(
        &self,
        pk: &HipProvingKey,
        record: &mut ExecutionRecord,
        challenger: &mut Challenger<SC>,
    ) -> Result<MachineProof<SC>, HipProverError>
    where
        A: for<'a> Air<DebugConstraintBuilder<'a, KoalaBear, <SC as StarkGenericConfig>::Challenge>>,
    {
        // prover.rs:560-582 with the trace generation moved to the device: the byte-lookup
        // multiplicities (generate_dependencies, prover.rs:570) are computed there from the same
        // events; the host record gets them too only where the debug builder reads them
        #[cfg(feature = "debug")]
        self.machine().generate_dependencies(record, None);
        pk.observe_into(challenger); // prover.rs:572
        // the compact hand-over (16 B per cycle), pipelined with its DMA; CycleArrays::new +
        // bfz_record_from_cycles and EventArrays + bfz_record_from_events remain for callers that
        // hold the cycles or the full event vectors
        let rec = HipRecord(CycleArrays::hand_over(pk.dev, record));
        let mut data = core::ptr::null_mut();
        let mut root = [0u32; 8];
        sys::check(unsafe {
            sys::bfz_record_main_commit(pk.dev, rec.0, &mut data, root.as_mut_ptr())
        });
        let main_commit = commitment(&root);
        // open reads the device data only: no host traces, chip ordering fixed by libbfz
        let data = ShardMainData::new(Vec::new(), main_commit, HipMainData(data), HashMap::new());
        let shard_proof = self.open(pk, data, &mut challenger.clone())?; // prover.rs:578
        drop(rec);
        Ok(MachineProof { shard_proof })
    }
}

impl HipProver {
    /// Pipelined proofs of one program over many inputs (bfz_prove_batch): execution and event
    /// upload of job k+1 run under the GPU proof of job k.  Returns the reference's ShardProof
    /// per input.
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
            .map(|(p, n)| Self::shard_proof(&unsafe { sys::take_bytes(p, n) }).expect("bincode"))
            .collect()
    }

    /// bfz_setup on the program text directly (a device key without the host StarkProvingKey;
    /// cached per program in libbfz).
    pub fn setup_device_only(&self, program: &Program) -> (*mut sys::bfz_pk, [u32; 8]) {
        let src = CString::new(program_source(program)).unwrap();
        let mut dev = core::ptr::null_mut();
        let mut root = [0u32; 8];
        sys::check(unsafe { sys::bfz_setup(src.as_ptr(), &mut dev, root.as_mut_ptr()) });
        (dev, root)
    }
}
