"""Random Brainfuck programs that halt (test helper shared by the CPU and GPU suites)."""


def random_program(rng, size, allow_negative=True):
    """A random balanced Brainfuck program that halts: loops always start with a '-' ... ']'
    body that decrements the cell it tests, over a bounded tape excursion (pointer-neutral).
    rng: a numpy Generator.  allow_negative=False never moves the memory pointer below cell 0:
    the reference's MemoryInstrs AIR range-checks the pointer as a KoalaBear word
    (memory/instructions/air.rs:37-61) while its executor wraps it as a u32
    (executor.rs:137-138), so a program that steps below 0 executes but has no valid proof."""
    out = []
    ptr = 0
    for _ in range(size):
        r = rng.random()
        if r < 0.25:
            out.append("+" * rng.integers(1, 6))
        elif r < 0.35:
            out.append("-")
        elif r < 0.55:
            step = ">" if rng.random() < 0.6 else "<"
            if step == "<" and ptr == 0 and not allow_negative:
                step = ">"
            ptr += 1 if step == ">" else -1
            out.append(step)
        elif r < 0.65:
            out.append(".")
        elif r < 0.7:
            out.append(",")
        else:
            k = int(rng.integers(1, 4))
            out.append("[-" + ">" * k + "+" + "<" * k + "]")
    return "".join(out)
