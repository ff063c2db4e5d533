"""Brainfuck guest programs (test/bench fixtures).

The first five are the reference's own guests (crates/test-artifacts/guests/*.bf, exposed as
FIBO_BF ... PRINTA_BF by crates/test-artifacts/src/lib.rs:1-5); examples/hello uses HELLO.

FIBO_X4 is this repo's 2^22-row workload: the reference fibonacci guest wrapped in an outer
loop that runs it 4 times (the guest reads its single input byte with ',', and the reference
executor never advances the input pointer, so every pass computes fib(n) again).  With
stdin [255] it executes 3,767,729 cycles, i.e. a 2^22-row Cpu trace (the reference guest
alone tops out at 941,747 cycles = 2^20 rows for n = 255).
"""

FIBO = ",>+>+<<[->>[->+>+<<]<[->>+<<]>>[-<+>]>[-<<<+>>>]<<<<]>>."
HELLO = ">++++++++[<+++++++++>-]<.>++++[<+++++++>-]<+.+++++++..+++.>>++++++[<+++++++>-]<+"
LOOP = "+++++[-]."
MOVE = ">>>>++.<<<<."
PRINTA = "+++++ +++++\n" * 6 + "+++++\n."  # 65 '+' -> 'A'

FIBO_X4 = "++++[>" + FIBO + "[-]<[-]<<-]"

# (program, stdin) pairs proven in the reference's test suite
# (crates/core/machine/src/brainfuck/mod.rs:113-189)
REFERENCE_PROGRAMS = [
    ("instructions", "+-><,.", [1]),
    ("add_sub", "++-", []),
    ("mem", ">><", []),
    ("jmp", "[----]", []),
    ("io", ",.", [1]),
    ("printa", PRINTA, []),
    ("move", MOVE, []),
    ("loop", LOOP, []),
    ("hello", HELLO, []),
    ("fibo17", FIBO, [17]),
]
