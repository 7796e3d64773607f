"""Lightning-free reader for the reference's `checkpoints/*.ckpt` state dicts.

The reference restores trained models with `*.load_from_checkpoint` (`data_utils.py:36-47`). Those
files are PyTorch zip archives: `archive/data.pkl` (a pickle) plus one raw little-endian storage per
tensor under `archive/data/<key>`. Un-pickling would execute code named by the file, so this reader
never does: it walks the pickle's opcode stream with `pickletools.genops` on a symbolic stack (globals
stay strings, calls stay tuples) and pulls out `state_dict` entries of the form
`_rebuild_tensor_v2(persistent_load(('storage', <type>, key, device, numel)), offset, size, stride)`.
Tensor bytes are then read straight out of the zip.
"""
from __future__ import annotations

import pickletools
import zipfile

import numpy as np

_DTYPES = {"FloatStorage": np.float32, "DoubleStorage": np.float64, "LongStorage": np.int64,
           "IntStorage": np.int32, "HalfStorage": np.float16, "BoolStorage": np.bool_}


class _Mark:
    pass


def _symbolic_unpickle(data: bytes):
    stack, memo, marks = [], {}, []

    def pop_mark():
        m = marks.pop()
        items = stack[m:]
        del stack[m:]
        return items

    for op, arg, _pos in pickletools.genops(data):
        name = op.name
        if name in ("PROTO", "FRAME"):
            continue
        if name == "STOP":
            break
        if name == "MARK":
            marks.append(len(stack))
        elif name in ("EMPTY_DICT",):
            stack.append({})
        elif name in ("EMPTY_LIST",):
            stack.append([])
        elif name in ("EMPTY_TUPLE",):
            stack.append(())
        elif name in ("SHORT_BINUNICODE", "BINUNICODE", "BINUNICODE8", "UNICODE", "SHORT_BINSTRING",
                      "BINSTRING", "STRING", "SHORT_BINBYTES", "BINBYTES", "BINBYTES8",
                      "BININT", "BININT1", "BININT2", "LONG1", "LONG4", "INT", "LONG",
                      "BINFLOAT", "FLOAT"):
            stack.append(arg)
        elif name == "NONE":
            stack.append(None)
        elif name == "NEWTRUE":
            stack.append(True)
        elif name == "NEWFALSE":
            stack.append(False)
        elif name == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif name == "TUPLE1":
            stack.append((stack.pop(),))
        elif name == "TUPLE2":
            b = stack.pop(); a = stack.pop(); stack.append((a, b))
        elif name == "TUPLE3":
            c = stack.pop(); b = stack.pop(); a = stack.pop(); stack.append((a, b, c))
        elif name == "LIST":
            stack.append(list(pop_mark()))
        elif name == "DICT":
            items = pop_mark()
            stack.append({items[i]: items[i + 1] for i in range(0, len(items), 2)})
        elif name == "GLOBAL":
            mod, _, qual = arg.partition(" ")
            stack.append(("global", mod, qual))
        elif name == "STACK_GLOBAL":
            qual = stack.pop(); mod = stack.pop(); stack.append(("global", mod, qual))
        elif name in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = stack[-1]
        elif name == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif name in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[arg])
        elif name == "SETITEM":
            v = stack.pop(); k = stack.pop()
            if isinstance(stack[-1], dict):
                stack[-1][k] = v
        elif name == "SETITEMS":
            items = pop_mark()
            if isinstance(stack[-1], dict):
                for i in range(0, len(items), 2):
                    stack[-1][items[i]] = items[i + 1]
        elif name == "APPEND":
            v = stack.pop()
            if isinstance(stack[-1], list):
                stack[-1].append(v)
        elif name == "APPENDS":
            items = pop_mark()
            if isinstance(stack[-1], list):
                stack[-1].extend(items)
        elif name == "REDUCE":
            args = stack.pop(); fn = stack.pop()
            if fn == ("global", "collections", "OrderedDict"):
                stack.append({})   # filled by the SETITEMS that follow
            else:
                stack.append(("call", fn, args))
        elif name in ("NEWOBJ",):
            args = stack.pop(); cls = stack.pop(); stack.append(("call", cls, args))
        elif name == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if isinstance(obj, tuple) and obj and obj[0] == "call":
                stack[-1] = obj + (("state", state),)
        elif name == "BINPERSID":
            stack.append(("persid", stack.pop()))
        elif name == "POP":
            stack.pop()
        elif name == "POP_MARK":
            pop_mark()
        elif name == "DUP":
            stack.append(stack[-1])
        else:
            raise ValueError(f"unsupported pickle opcode {name}")
    return stack[-1] if stack else None


def _as_tensor_spec(v):
    """('call', ('global','torch._utils','_rebuild_tensor_v2'), (persid, offset, size, stride, ...))"""
    if not (isinstance(v, tuple) and len(v) >= 3 and v[0] == "call"):
        return None
    fn, args = v[1], v[2]
    if not (isinstance(fn, tuple) and fn[:1] == ("global",) and fn[2] == "_rebuild_tensor_v2"):
        return None
    pers, offset, size, stride = args[0], args[1], args[2], args[3]
    ident = pers[1]
    _, stype, key, _device, _numel = ident
    dtype = _DTYPES[stype[2]] if isinstance(stype, tuple) else np.float32
    return key, dtype, int(offset), tuple(size), tuple(stride)


def _check_view(name, numel: int, offset: int, size, stride):
    """Bounds of a (offset, size, stride) view of a storage of `numel` elements, checked before
    as_strided touches memory: a malformed or hostile pickle must not read outside the buffer."""
    if len(size) != len(stride):
        raise ValueError(f"{name}: size {size} and stride {stride} differ in rank")
    if offset < 0 or any(s < 0 for s in size) or any(st < 0 for st in stride):
        raise ValueError(f"{name}: negative offset/size/stride ({offset}, {size}, {stride})")
    if any(s == 0 for s in size):
        if offset > numel:
            raise ValueError(f"{name}: offset {offset} past storage of {numel} elements")
        return
    last = offset + sum((s - 1) * st for s, st in zip(size, stride))
    if last >= numel:
        raise ValueError(f"{name}: view reaches element {last}, storage holds {numel}")


def read_state_dict(path: str) -> dict:
    """{name: np.ndarray} for every tensor in the checkpoint's `state_dict` (copies, C-order)."""
    with zipfile.ZipFile(path) as zf:
        names = zf.namelist()
        root = names[0].split("/")[0]
        obj = _symbolic_unpickle(zf.read(f"{root}/data.pkl"))
        sd = obj.get("state_dict", obj) if isinstance(obj, dict) else None
        if not isinstance(sd, dict):
            # OrderedDict is pickled as REDUCE(OrderedDict, ()) + SETITEMS -> our call tuple
            raise ValueError("no state_dict found")
        if isinstance(sd, tuple):
            raise ValueError("unexpected state_dict encoding")
        out = {}
        for name, v in sd.items() if isinstance(sd, dict) else []:
            spec = _as_tensor_spec(v)
            if spec is None:
                continue
            key, dtype, offset, size, stride = spec
            raw = np.frombuffer(zf.read(f"{root}/data/{key}"), dtype=dtype)
            itemsize = np.dtype(dtype).itemsize
            _check_view(name, raw.size, offset, size, stride)
            arr = np.lib.stride_tricks.as_strided(
                raw[offset:], shape=size, strides=tuple(s * itemsize for s in stride),
                writeable=False)
            out[name] = np.ascontiguousarray(arr)
        return out
