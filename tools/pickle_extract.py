#!/usr/bin/env python3
"""No-code reader for the reference's pandas pickles (build container only).

``age_ens_runs_mcmc/C_in_dict.pk`` and ``map_dict.pk`` (written by
age_modeling_mcmc.prep.py:216-219 and :491-500) are pickles of dicts of pandas
DataFrames.  Loading a pickle executes whatever callables it names, so this module
never unpickles: it walks the opcode stream with ``pickletools.genops`` and runs a
*symbolic* stack machine over it.  GLOBAL / REDUCE / NEWOBJ / BUILD produce inert
records (``Global``, ``Call``) -- nothing is imported, looked up or called.  Only
plain values (str, int, float, bytes, tuples, lists, dicts as pair lists) are
materialised.

The float64 / int64 block buffers of every ``numpy.core.multiarray._reconstruct``
record are then decoded with ``numpy.frombuffer`` (dtype and shape taken from the
record's own state tuple), and each DataFrame is rebuilt as
``{"columns": [...], "index": ndarray, "values": ndarray [n_cols][n_rows]}``.
"""
import pickletools

import numpy as np


class Global:
    def __init__(self, module, name):
        self.module, self.name = module, name

    @property
    def qual(self):
        return self.module + "." + self.name

    def __repr__(self):
        return "Global(%s)" % self.qual


class Call:
    """func(*args) or cls.__new__(cls, *args), plus the state a BUILD attached."""

    def __init__(self, func, args):
        self.func, self.args, self.state = func, args, None

    def __repr__(self):
        return "Call(%r, %r%s)" % (self.func, self.args, ", state" if self.state is not None else "")


class PDict:
    """A pickled dict as an ordered list of (key, value) pairs (keys may be records)."""

    def __init__(self):
        self.items = []

    def get(self, key, default=None):
        for k, v in self.items:
            if k == key:
                return v
        return default


_MARK = object()


def symbolic_load(data):
    """Run the opcode stream symbolically; returns the top-level record."""
    stack, memo = [], {}

    def pop_mark():
        i = len(stack) - 1
        while stack[i] is not _MARK:
            i -= 1
        items = stack[i + 1:]
        del stack[i:]
        return items

    for op, arg, _pos in pickletools.genops(data):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        if n == "STOP":
            break
        if n == "MARK":
            stack.append(_MARK)
        elif n in ("SHORT_BINUNICODE", "BINUNICODE", "BINUNICODE8", "UNICODE", "SHORT_BINSTRING", "BINSTRING"):
            stack.append(arg)
        elif n in ("SHORT_BINBYTES", "BINBYTES", "BINBYTES8"):
            stack.append(bytes(arg))
        elif n in ("BININT", "BININT1", "BININT2", "LONG1", "LONG4", "INT", "LONG"):
            stack.append(int(arg))
        elif n in ("BINFLOAT", "FLOAT"):
            stack.append(float(arg))
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "TUPLE1":
            stack[-1:] = [tuple(stack[-1:])]
        elif n == "TUPLE2":
            stack[-2:] = [tuple(stack[-2:])]
        elif n == "TUPLE3":
            stack[-3:] = [tuple(stack[-3:])]
        elif n == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif n == "EMPTY_LIST":
            stack.append([])
        elif n == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif n == "APPENDS":
            items = pop_mark()
            stack[-1].extend(items)
        elif n == "EMPTY_DICT":
            stack.append(PDict())
        elif n == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1].items.append((k, v))
        elif n == "SETITEMS":
            items = pop_mark()
            d = stack[-1]
            for i in range(0, len(items), 2):
                d.items.append((items[i], items[i + 1]))
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[int(arg)] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[int(arg)])
        elif n == "STACK_GLOBAL":
            name = stack.pop()
            module = stack.pop()
            stack.append(Global(module, name))
        elif n == "GLOBAL":
            module, name = arg.split(" ", 1)
            stack.append(Global(module, name))
        elif n == "REDUCE":
            args = stack.pop()
            func = stack.pop()
            stack.append(Call(func, args))
        elif n == "NEWOBJ":
            args = stack.pop()
            cls = stack.pop()
            stack.append(Call(cls, args))
        elif n == "BUILD":
            state = stack.pop()
            stack[-1].state = state
        else:
            raise ValueError("opcode %s not handled by the symbolic reader" % n)
    if len(stack) != 1:
        raise ValueError("malformed pickle: %d items left on the stack" % len(stack))
    return stack[0]


def as_ndarray(rec):
    """numpy.core.multiarray._reconstruct record -> ndarray (numeric) or list (object)."""
    if not (isinstance(rec, Call) and isinstance(rec.func, Global) and rec.func.name == "_reconstruct"):
        raise ValueError("not an ndarray record: %r" % (rec,))
    _ver, shape, dt, fortran, raw = rec.state
    code = dt.args[0]
    if code == "O8":
        return list(raw)
    byteorder = dt.state[1]
    arr = np.frombuffer(raw, dtype=np.dtype((byteorder if byteorder in "<>" else "=") + code))
    return arr.reshape(shape, order="F" if fortran else "C").copy()


def as_index(rec):
    """pandas Index record (_new_Index(cls, {'data': ndarray, 'name': ...}) or RangeIndex)."""
    if isinstance(rec, Call) and isinstance(rec.func, Global) and rec.func.name == "_new_Index":
        cls, d = rec.args
        if cls.name == "RangeIndex":
            return np.arange(d.get("start"), d.get("stop"), d.get("step")), d.get("name")
        return as_ndarray(d.get("data")), d.get("name")
    raise ValueError("not an Index record: %r" % (rec,))


def as_frame(rec):
    """DataFrame record -> dict(columns, index, index_name, values [n_cols][n_rows])."""
    mgr = rec.state.get("_mgr")
    blocks, axes = mgr.args
    columns, _ = as_index(axes[0])
    index, index_name = as_index(axes[1])
    values = np.full((len(columns), len(index)), np.nan)
    for blk in blocks:
        arr = as_ndarray(blk.args[0])                 # [n_block_cols][n_rows]
        sl = blk.args[1]                              # builtins.slice(start, stop, step)
        if isinstance(sl, Call) and sl.func.name == "slice":
            start, stop, step = sl.args
            cols = range(start, stop, step or 1)
        else:
            cols = list(as_ndarray(sl))
        for j, c in enumerate(cols):
            values[c] = arr[j]
    return {"columns": list(columns), "index": np.asarray(index), "index_name": index_name, "values": values}


def read_frame_dict(path):
    """{key: frame dict} of a pickled dict of DataFrames, read without unpickling."""
    with open(path, "rb") as f:
        top = symbolic_load(f.read())
    return {k: as_frame(v) for k, v in top.items}


if __name__ == "__main__":
    import sys
    for p in sys.argv[1:]:
        for k, fr in read_frame_dict(p).items():
            print(p, k, fr["columns"], fr["index_name"], fr["index"][:3], fr["index"][-3:], fr["values"].shape,
                  fr["values"][:, -3:].tolist())
