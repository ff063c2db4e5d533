/* ORACLE — test infrastructure only.  BF executor, chip traces, lookups, AIR constraints. */
#ifndef OR_MACHINE_H
#define OR_MACHINE_H
#include "or_field.h"

/* Opcode values (crates/core/executor/src/opcode.rs:10-27). */
enum { OP_LOOP_START = 0, OP_LOOP_END = 1, OP_ADD = 2, OP_SUB = 3, OP_FWD = 4, OP_BWD = 5,
       OP_INPUT = 6, OP_OUTPUT = 7 };

typedef struct { int opcode; uint32_t op_a; } or_instr;
typedef struct { or_instr* ins; size_t n; } or_program;

/* MemoryRecordEnum: kind 0 = none, 1 = read, 2 = write. */
typedef struct { int kind; uint8_t value, prev_value; uint32_t ts, prev_ts; } or_memacc;
typedef struct {
  uint32_t clk, pc, next_pc, mp, next_mp;
  uint8_t mv, next_mv;
  or_memacc mv_access, next_mv_access;
} or_cpu_ev;
typedef struct { uint32_t pc; int opcode; uint8_t next_mv, mv; } or_alu_ev;
typedef struct { uint32_t pc, next_pc; int opcode; uint32_t dst; uint8_t mv; } or_jump_ev;
typedef struct { uint32_t clk, pc; int opcode; uint32_t mp, next_mp; } or_meminstr_ev;
typedef struct { uint32_t pc; int opcode; uint32_t mp; uint8_t mv; } or_io_ev;
typedef struct { uint32_t addr, init_ts, final_ts; uint8_t init_v, final_v; } or_mem_ev;

typedef struct {
  or_program prog;
  or_cpu_ev* cpu; size_t ncpu;
  or_alu_ev* alu; size_t nalu;
  or_jump_ev* jump; size_t njump;
  or_meminstr_ev* mi; size_t nmi;
  or_io_ev* io; size_t nio;
  or_mem_ev* mem; size_t nmem;
  uint64_t* u8_mult;  /* [256]   U8Range multiplicities   */
  uint64_t* u16_mult; /* [65536] U16Range multiplicities  */
  uint8_t* output; size_t noutput;
  uint64_t global_clk;
  uint32_t final_pc, final_mp;
} or_record;

int or_parse_program(const char* src, or_program* p);
int or_execute(const or_program* p, const uint8_t* in, size_t nin, or_record* r);
void or_generate_dependencies(or_record* r);
void or_record_free(or_record* r);

/* Chips in machine order (crates/core/machine/src/brainfuck/mod.rs:53-81). */
enum { CHIP_CPU = 0, CHIP_PROGRAM, CHIP_ADDSUB, CHIP_JUMP, CHIP_MEMORY, CHIP_BYTE,
       CHIP_MEMINSTRS, CHIP_IO, NUM_CHIPS };

typedef struct {
  const char* name;
  int main_w, prep_w, local_only;
} or_chip_info;
extern const or_chip_info OR_CHIPS[NUM_CHIPS];

int or_chip_included(int chip, const or_record* r);
/* Main trace (row-major, canonical). Returns height; *out malloc'd. */
size_t or_main_trace(int chip, const or_record* r, fp** out);
/* Preprocessed trace for Program/Byte; returns height or 0. */
size_t or_prep_trace(int chip, const or_program* p, fp** out);

/* Lookups: affine combos of (prep|main) columns. */
typedef struct { int n; int src[8]; int col[8]; fp w[8]; fp c; } or_vcol;
typedef struct { int kind; int nvals; or_vcol vals[8]; or_vcol mult; } or_lookup;
typedef struct { int nsends, nrecvs; or_lookup sends[16], recvs[16]; } or_chip_lookups;
void or_chip_lookups_get(int chip, or_chip_lookups* out);
int or_perm_width(int chip); /* in EF columns */

/* Constraint folder (ProverConstraintFolder / VerifierConstraintFolder semantics). */
typedef struct {
  const ef *prep_l, *prep_n, *main_l, *main_n, *perm_l, *perm_n;
  ef perm_alpha, perm_beta, cumsum;
  ef is_first, is_last, is_trans;
  ef alpha, acc;
} or_folder;
void or_eval_chip(int chip, or_folder* f);

#endif
