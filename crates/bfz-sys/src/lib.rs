//! Raw bindings of `include/bfz.h` (the C ABI of the MI355X core prover).  One declaration per
//! header entry point, same names and argument order; field data is `u32` in Montgomery form,
//! i.e. the in-memory layout of `[KoalaBear]` (p3 `MontyField31`).
#![allow(non_camel_case_types)]
use core::ffi::c_void;
use std::os::raw::{c_char, c_int};

#[repr(C)]
pub struct bfz_pk {
    _opaque: [u8; 0],
}
#[repr(C)]
pub struct bfz_record {
    _opaque: [u8; 0],
}
#[repr(C)]
pub struct bfz_main_data {
    _opaque: [u8; 0],
}
#[repr(C)]
pub struct bfz_cycle_upload {
    _opaque: [u8; 0],
}

/// p3 `DuplexChallenger<KoalaBear, Poseidon2KoalaBear<16>, 16, 8>` as plain data.
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct bfz_challenger {
    pub sponge_state: [u32; 16],
    pub input_buffer: [u32; 8],
    pub n_input: u32,
    pub output_buffer: [u32; 8],
    pub n_output: u32,
}

#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct bfz_timings {
    pub trace_ms: f64,
    pub main_commit_ms: f64,
    pub perm_ms: f64,
    pub quotient_ms: f64,
    pub open_ms: f64,
    pub fri_ms: f64,
    pub total_ms: f64,
    pub lde_ms: f64,
    pub lde_bytes: f64,
    pub lde_calls: c_int,
    pub ntt_kernel_ms: f64,
    pub ntt_kernel_bytes: f64,
    pub ntt_kernel_launches: c_int,
    pub p2_kernel_ms: f64,
    pub p2_perms: f64,
    pub p2_launches: c_int,
    pub lde_elem_stages: f64,
    pub open_kernel_ms: f64,
    pub open_kernel_bytes: f64,
    pub open_kernel_launches: c_int,
    pub reduce_kernel_ms: f64,
    pub reduce_kernel_bytes: f64,
    pub reduce_kernel_launches: c_int,
    pub perm_rows_ms: f64,
    pub perm_idft_ms: f64,
    pub perm_dft_ms: f64,
    pub perm_hash_ms: f64,
    pub main_idft_ms: f64,
    pub main_dft_ms: f64,
    pub main_hash_ms: f64,
    pub main_cells: f64,
    pub perm_cells: f64,
}

#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct bfz_batch_stats {
    pub wall_ms: f64,
    pub exec_ms: f64,
    pub upload_ms: f64,
    pub prove_ms: f64,
    pub exec_threads: c_int,
}

/// `Option<MemoryRecordEnum>` (events/memory.rs:31-79): kind 0 = None, 1 = Read, 2 = Write.
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct bfz_memory_access {
    pub kind: u8,
    pub value: u8,
    pub prev_value: u8,
    pub _pad: u8,
    pub timestamp: u32,
    pub prev_timestamp: u32,
}
/// `CpuEvent` (events/cpu.rs).
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct bfz_cpu_event {
    pub clk: u32,
    pub pc: u32,
    pub next_pc: u32,
    pub mp: u32,
    pub next_mp: u32,
    pub mv: u8,
    pub next_mv: u8,
    pub _pad: [u8; 2],
    pub mv_access: bfz_memory_access,
    pub next_mv_access: bfz_memory_access,
}
/// `AluEvent` (events/instr.rs).
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct bfz_alu_event {
    pub pc: u32,
    pub opcode: u8,
    pub next_mv: u8,
    pub mv: u8,
    pub _pad: u8,
}
/// `JumpEvent`.
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct bfz_jump_event {
    pub pc: u32,
    pub next_pc: u32,
    pub opcode: u8,
    pub _pad: [u8; 3],
    pub dst: u32,
    pub mv: u8,
    pub _pad2: [u8; 3],
}
/// `MemInstrEvent`.
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct bfz_mem_instr_event {
    pub clk: u32,
    pub pc: u32,
    pub opcode: u8,
    pub _pad: [u8; 3],
    pub mp: u32,
    pub next_mp: u32,
}
/// `IoEvent`.
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct bfz_io_event {
    pub pc: u32,
    pub opcode: u8,
    pub _pad: [u8; 3],
    pub mp: u32,
    pub mv: u8,
    pub _pad2: [u8; 3],
}
/// `MemoryEvent` (addr, initial_mem_access, final_mem_access).
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct bfz_memory_event {
    pub addr: u32,
    pub initial_timestamp: u32,
    pub final_timestamp: u32,
    pub initial_value: u8,
    pub final_value: u8,
    pub _pad: [u8; 2],
}
/// One `CpuEvent` in the compact hand-over of `bfz_record_from_cycles` (16 bytes): the rest of
/// the record is rebuilt on the device (include/bfz.h).
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct bfz_cycle {
    pub pc: u32,
    pub mp: u32,
    pub prev_ts: u32,
    pub mv: u8,
    pub prev_value: u8,
    pub _pad: [u8; 2],
}
/// The `ExecutionRecord` event vectors (record.rs:15-34) as pointer + length pairs.
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct bfz_events {
    pub cpu: *const bfz_cpu_event,
    pub n_cpu: usize,
    pub add: *const bfz_alu_event,
    pub n_add: usize,
    pub sub: *const bfz_alu_event,
    pub n_sub: usize,
    pub jump: *const bfz_jump_event,
    pub n_jump: usize,
    pub io: *const bfz_io_event,
    pub n_io: usize,
    pub memory_instr: *const bfz_mem_instr_event,
    pub n_memory_instr: usize,
    pub memory: *const bfz_memory_event,
    pub n_memory: usize,
}

pub type bfz_allgather_fn =
    Option<unsafe extern "C" fn(ctx: *mut c_void, send: *const c_void, bytes: usize, recv: *mut c_void) -> c_int>;
pub type bfz_allreduce_u32_fn = Option<unsafe extern "C" fn(ctx: *mut c_void, data: *mut u32, n: usize) -> c_int>;
pub type bfz_alltoall_fn = Option<unsafe extern "C" fn(ctx: *mut c_void) -> c_int>;

#[link(name = "bfz")]
extern "C" {
    pub fn bfz_init(device: c_int) -> c_int;
    pub fn bfz_last_error() -> *const c_char;
    pub fn bfz_build_id() -> *const c_char;
    pub fn bfz_device_name(buf: *mut c_char, cap: usize) -> c_int;
    pub fn bfz_free(p: *mut c_void);
    pub fn bfz_synchronize() -> c_int;
    pub fn bfz_selftest(name: *const c_char) -> c_int;

    pub fn bfz_execute(elf: *const c_char, stdin_data: *const u8, nin: usize, out: *mut u8,
                       out_cap: usize, out_len: *mut usize, cycles: *mut u64) -> c_int;
    pub fn bfz_trace(elf: *const c_char, stdin_data: *const u8, nin: usize, chip: c_int, prep: c_int,
                     out: *mut *mut u32, height: *mut usize, width: *mut usize) -> c_int;
    pub fn bfz_execute_events(elf: *const c_char, stdin_data: *const u8, nin: usize, executor: c_int,
                              out: *mut *mut u8, out_len: *mut usize) -> c_int;
    pub fn bfz_perm_trace(chip: c_int, main: *const u32, prep: *const u32, height: usize,
                          alpha: *const u32, beta: *const u32, out: *mut *mut u32,
                          width: *mut usize, cumsum: *mut u32) -> c_int;
    pub fn bfz_trace_device(elf: *const c_char, stdin_data: *const u8, nin: usize, chip: c_int,
                            out: *mut *mut u32, height: *mut usize, width: *mut usize) -> c_int;

    pub fn bfz_setup(elf: *const c_char, pk: *mut *mut bfz_pk, vk_commit: *mut u32) -> c_int;
    pub fn bfz_pk_free(pk: *mut bfz_pk);
    pub fn bfz_pk_from_host(chips: *const c_int, traces: *const *const u32, heights: *const usize,
                            widths: *const usize, n: usize, commit: *const u32,
                            pk: *mut *mut bfz_pk) -> c_int;
    pub fn bfz_pk_commit(pk: *const bfz_pk, commit: *mut u32) -> c_int;

    pub fn bfz_main_commit(pk: *const bfz_pk, chips: *const c_int, traces: *const *const u32,
                           heights: *const usize, widths: *const usize, nchips: usize,
                           out: *mut *mut bfz_main_data, root: *mut u32) -> c_int;
    pub fn bfz_record_main_commit(pk: *const bfz_pk, rec: *const bfz_record,
                                  out: *mut *mut bfz_main_data, root: *mut u32) -> c_int;
    pub fn bfz_challenger_observe_pk(pk: *const bfz_pk, ch: *mut bfz_challenger) -> c_int;
    pub fn bfz_open(pk: *const bfz_pk, data: *mut bfz_main_data, ch: *mut bfz_challenger,
                    proof: *mut *mut u8, proof_len: *mut usize) -> c_int;
    pub fn bfz_main_data_free(data: *mut bfz_main_data);

    pub fn bfz_prove(pk: *const bfz_pk, stdin_data: *const u8, nin: usize, proof: *mut *mut u8,
                     proof_len: *mut usize) -> c_int;
    pub fn bfz_prove_traces(pk: *const bfz_pk, chips: *const c_int, traces: *const *const u32,
                            heights: *const usize, widths: *const usize, nchips: usize,
                            proof: *mut *mut u8, proof_len: *mut usize) -> c_int;
    pub fn bfz_verify(elf: *const c_char, vk_commit: *const u32, proof: *const u8,
                      proof_len: usize) -> c_int;
    pub fn bfz_prove_batch(pk: *const bfz_pk, stdins: *const *const u8, nins: *const usize,
                           njobs: usize, exec_threads: c_int, proofs: *mut *mut u8,
                           proof_lens: *mut usize, stats: *mut bfz_batch_stats) -> c_int;

    pub fn bfz_record_new(pk: *const bfz_pk, stdin_data: *const u8, nin: usize,
                          rec: *mut *mut bfz_record, cycles: *mut u64) -> c_int;
    pub fn bfz_record_prove(pk: *const bfz_pk, rec: *const bfz_record, proof: *mut *mut u8,
                            proof_len: *mut usize, timings: *mut bfz_timings) -> c_int;
    pub fn bfz_record_free(rec: *mut bfz_record);
    pub fn bfz_record_from_events(pk: *const bfz_pk, events: *const bfz_events,
                                  rec: *mut *mut bfz_record) -> c_int;
    pub fn bfz_record_from_cycles(pk: *const bfz_pk, cycles: *const bfz_cycle, n_cycles: usize,
                                  memory: *const bfz_memory_event, n_memory: usize,
                                  rec: *mut *mut bfz_record) -> c_int;
    pub fn bfz_cycles_begin(pk: *const bfz_pk, n_cycles: usize, up: *mut *mut bfz_cycle_upload) -> c_int;
    pub fn bfz_cycles_push(up: *mut bfz_cycle_upload, first: usize, cycles: *const bfz_cycle,
                           n: usize) -> c_int;
    pub fn bfz_cycles_finish(up: *mut bfz_cycle_upload, memory: *const bfz_memory_event,
                             n_memory: usize, rec: *mut *mut bfz_record) -> c_int;
    pub fn bfz_cycles_abort(up: *mut bfz_cycle_upload);
    pub fn bfz_host_alloc(bytes: usize, out: *mut *mut c_void) -> c_int;
    pub fn bfz_host_free(p: *mut c_void);
    pub fn bfz_record_prove_repeat(pk: *const bfz_pk, rec: *const bfz_record, count: c_int,
                                   inflight: c_int, proof: *mut *mut u8, len: *mut usize,
                                   wall_ms: *mut f64) -> c_int;
    pub fn bfz_record_prove_sharded(pk: *const bfz_pk, rec: *const bfz_record, rank: c_int,
                                    world: c_int, allgather: bfz_allgather_fn,
                                    allreduce_sum: bfz_allreduce_u32_fn, ctx: *mut c_void,
                                    proof: *mut *mut u8, proof_len: *mut usize,
                                    timings: *mut bfz_timings) -> c_int;
    pub fn bfz_record_prove_shard_solo(pk: *const bfz_pk, rec: *const bfz_record, rank: c_int,
                                       world: c_int, timings: *mut bfz_timings) -> c_int;
    pub fn bfz_shard_solo_exchanges(kinds: *mut c_int, bytes: *mut u64, cap: usize, n: *mut usize) -> c_int;
    pub fn bfz_shard_solo_overlaps(ms: *mut f64, cap: usize, n: *mut usize) -> c_int;
    pub fn bfz_device_pool_bytes(lane: c_int, bytes: *mut u64) -> c_int;
    pub fn bfz_commit_fri_sharded(d_cols: *const u32, log_n: c_int, w_local: usize, rank: c_int,
                                  world: c_int, d_send: *mut u32, d_recv: *mut u32,
                                  alltoall: bfz_alltoall_fn, allgather: bfz_allgather_fn,
                                  ctx: *mut c_void, out: *mut u32, cap: usize,
                                  nwords: *mut usize) -> c_int;

    pub fn bfz_set_num_queries(num_queries: c_int) -> c_int;
    pub fn bfz_set_pcs_variant(observe_openings: c_int) -> c_int;
    /// Test-only fault injection (bit 0: perturb the device challenger); 0 = off.
    pub fn bfz_set_fault_injection(mask: c_int) -> c_int;

    pub fn bfz_proof_to_bincode(proof: *const u8, len: usize, field_repr: c_int, out: *mut *mut u8,
                                out_len: *mut usize) -> c_int;
    pub fn bfz_proof_from_bincode(bytes: *const u8, len: usize, field_repr: c_int, out: *mut *mut u8,
                                  out_len: *mut usize) -> c_int;
    pub fn bfz_verify_bincode(elf: *const c_char, vk_commit: *const u32, bytes: *const u8,
                              len: usize, field_repr: c_int) -> c_int;

    pub fn bfz_coset_lde(evals: *const u32, n: usize, w: usize, shift: u32, lde_out: *mut u32) -> c_int;
    pub fn bfz_commit(mats: *const *const u32, heights: *const usize, widths: *const usize,
                      nmats: usize, root: *mut u32) -> c_int;
    pub fn bfz_poseidon2_permute(states: *mut u32, n: usize) -> c_int;
    pub fn bfz_poseidon2_permute_small(states: *mut u32, n: usize) -> c_int;
}

/// The message of the last failed call on this thread.
pub fn last_error() -> String {
    unsafe {
        let p = bfz_last_error();
        if p.is_null() {
            return String::new();
        }
        std::ffi::CStr::from_ptr(p).to_string_lossy().into_owned()
    }
}

/// Panics with the library's message on a non-zero status (the reference unwraps in the same
/// places, so a failing proof panics there too).
pub fn check(status: c_int) {
    if status != 0 {
        panic!("bfz status {status}: {}", last_error());
    }
}

/// Takes ownership of a malloc'd byte buffer returned by the library.
pub unsafe fn take_bytes(p: *mut u8, len: usize) -> Vec<u8> {
    let v = std::slice::from_raw_parts(p, len).to_vec();
    bfz_free(p as *mut c_void);
    v
}
