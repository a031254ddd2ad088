"""A small evaluator for the table-driven Go unit tests of the reference, used ONLY to
transcribe their test tables (inputs + expected outputs) into JSON fixtures.

It reads the reference's *_test.go files as text (study), parses the subset of Go the
test tables are written in -- composite literals, the st.MakePod()/st.MakeNode()/
st.MakeLabelSelector() builder chains (pkg/scheduler/testing/wrappers.go), local variables,
one-line helper functions -- and evaluates them into v1 JSON objects.  Nothing of the
reference is executed or copied into the repository: the output is data.
"""
import re

# --------------------------------------------------------------------------------------
# tokenizer
# --------------------------------------------------------------------------------------
TOKEN = re.compile(r"""
    (?P<ws>\s+)|
    (?P<lc>//[^\n]*)|
    (?P<bc>/\*.*?\*/)|
    (?P<raw>`[^`]*`)|
    (?P<str>"(?:\\.|[^"\\])*")|
    (?P<num>\d+(?:\.\d+)?(?:[eE][+-]?\d+)?)|
    (?P<id>[A-Za-z_][A-Za-z_0-9]*)|
    (?P<op>:=|\.\.\.|&&|\|\||==|!=|<=|>=|<<|>>|[{}()\[\],:;.&*+\-/=<>!%])
""", re.S | re.X)


def tokenize(src):
    """Tokens with Go's automatic semicolon insertion (a newline after an identifier,
    literal, `)`, `]` or `}` ends the statement)."""
    out = []
    for m in TOKEN.finditer(src):
        k = m.lastgroup
        v = m.group()
        if k in ("ws", "lc", "bc"):
            if "\n" in v and out:
                last = out[-1]
                if last[0] in ("id", "str", "num") or last[1] in (")", "]", "}"):
                    out.append(("op", ";"))
            continue
        if k == "raw":
            out.append(("str", v[1:-1]))
        elif k == "str":
            out.append(("str", bytes(v[1:-1], "utf-8").decode("unicode_escape")))
        elif k == "num":
            out.append(("num", float(v) if "." in v or "e" in v.lower() else int(v)))
        else:
            out.append((k, v))
    out.append(("eof", None))
    return out


# --------------------------------------------------------------------------------------
# AST (tuples) + parser for the expression subset
# --------------------------------------------------------------------------------------
class Parser:
    def __init__(self, toks, i=0):
        self.t = toks
        self.i = i

    def peek(self, k=0):
        return self.t[self.i + k]

    def next(self):
        tok = self.t[self.i]
        self.i += 1
        return tok

    def accept(self, v):
        if self.t[self.i][1] == v and self.t[self.i][0] in ("op", "id"):
            self.i += 1
            return True
        return False

    def expect(self, v):
        tok = self.next()
        if tok[1] != v:
            raise SyntaxError(f"expected {v!r} got {tok!r} at {self.i}")
        return tok

    # ---- types ----
    def parse_type(self):
        if self.accept("*"):
            return ("ptr", self.parse_type())
        if self.peek()[1] == "[":
            self.next()
            if self.accept("]"):
                return ("slice", self.parse_type())
            n = self.parse_expr()
            self.expect("]")
            return ("array", n, self.parse_type())
        if self.accept("map"):
            self.expect("[")
            k = self.parse_type()
            self.expect("]")
            return ("map", k, self.parse_type())
        if self.accept("struct"):
            self.expect("{")
            depth = 1
            fields = []
            while depth:
                tok = self.next()
                if tok[1] == "{":
                    depth += 1
                elif tok[1] == "}":
                    depth -= 1
                elif depth == 1 and tok[0] == "id" and self.peek()[0] in ("id", "op"):
                    fields.append(tok[1])
            return ("struct", fields)
        if self.accept("func"):
            self.skip_parens()
            while self.peek()[1] not in ("{", ",", ")", "}"):
                self.next()
            return ("functype",)
        name = self.next()[1]
        while self.peek()[1] == "." and self.peek(1)[0] == "id":
            self.next()
            name += "." + self.next()[1]
        if self.peek()[1] == "[" and self.peek(1)[0] == "id" and self.peek(2)[1] == "]":  # generic instantiation
            self.next()
            self.next()
            self.next()
        return ("named", name)

    def skip_parens(self):
        self.expect("(")
        depth = 1
        while depth:
            tok = self.next()
            if tok[1] == "(":
                depth += 1
            elif tok[1] == ")":
                depth -= 1

    def skip_block(self):
        self.expect("{")
        depth = 1
        while depth:
            tok = self.next()
            if tok[1] == "{":
                depth += 1
            elif tok[1] == "}":
                depth -= 1

    # ---- expressions ----
    def parse_expr(self):
        return self.parse_binary(0)

    PREC = {"||": 1, "&&": 2, "==": 3, "!=": 3, "<": 3, "<=": 3, ">": 3, ">=": 3,
            "+": 4, "-": 4, "*": 5, "/": 5, "%": 5, "<<": 5, ">>": 5}

    def parse_binary(self, minp):
        left = self.parse_unary()
        while True:
            tok = self.peek()
            p = self.PREC.get(tok[1]) if tok[0] == "op" else None
            if p is None or p <= minp:
                return left
            self.next()
            right = self.parse_binary(p)
            left = ("bin", tok[1], left, right)

    def parse_unary(self):
        if self.accept("&"):
            return ("addr", self.parse_unary())
        if self.accept("-"):
            return ("neg", self.parse_unary())
        if self.accept("!"):
            return ("not", self.parse_unary())
        if self.peek()[1] == "*":
            self.next()
            return ("deref", self.parse_unary())
        return self.parse_postfix(self.parse_primary())

    def parse_primary(self):
        tok = self.peek()
        if tok[0] == "str":
            self.next()
            return ("lit", tok[1])
        if tok[0] == "num":
            self.next()
            return ("lit", tok[1])
        if tok[1] == "(":
            self.next()
            e = self.parse_expr()
            self.expect(")")
            return e
        if tok[1] in ("[", "map", "struct"):
            typ = self.parse_type()
            if self.peek()[1] == "{":
                return ("composite", typ, self.parse_elements())
            return ("type", typ)
        if tok[1] == "func":
            self.next()
            self.skip_parens()
            while self.peek()[1] != "{":
                self.next()
            self.skip_block()
            return ("unknown", "funclit")
        if tok[0] == "id":
            self.next()
            return ("id", tok[1])
        raise SyntaxError(f"unexpected {tok!r} at {self.i}")

    def parse_elements(self):
        self.expect("{")
        elems = []
        while not self.accept("}"):
            if self.peek()[1] == "{":
                val = ("elided", self.parse_elements())
            else:
                val = self.parse_expr()
            if self.accept(":"):
                key = val
                if self.peek()[1] == "{":
                    val = ("elided", self.parse_elements())
                else:
                    val = self.parse_expr()
                elems.append((key, val))
            else:
                elems.append((None, val))
            if not self.accept(","):
                self.expect("}")
                break
        return elems

    def parse_postfix(self, e):
        while True:
            tok = self.peek()
            if tok[1] == "." and self.peek(1)[0] == "id":
                self.next()
                e = ("sel", e, self.next()[1])
            elif tok[1] == "(":
                self.next()
                args = []
                while not self.accept(")"):
                    args.append(self.parse_expr())
                    self.accept("...")
                    if not self.accept(","):
                        self.expect(")")
                        break
                e = ("call", e, args)
            elif tok[1] == "[":
                # index or generic instantiation: f[T](x)
                self.next()
                if self.peek()[0] == "id" and self.peek(1)[1] == "]" and self.peek(2)[1] == "(":
                    self.next()
                    self.next()
                    continue
                idx = self.parse_expr()
                self.expect("]")
                e = ("index", e, idx)
            elif tok[1] == "{" and e[0] in ("id", "sel"):
                e = ("composite", ("named", _dotted(e)), self.parse_elements())
            else:
                return e


def _dotted(e):
    if e[0] == "id":
        return e[1]
    if e[0] == "sel":
        return _dotted(e[1]) + "." + e[2]
    raise ValueError(e)


def _looks_like_type(e):
    try:
        name = _dotted(e)
    except ValueError:
        return False
    last = name.split(".")[-1]
    return last[:1].isupper() and name.split(".")[0] in TYPE_PKGS


TYPE_PKGS = {"v1", "metav1", "fwk", "framework", "config", "resource", "st", "schema"}


# --------------------------------------------------------------------------------------
# file-level scan: package vars, helper funcs, test functions
# --------------------------------------------------------------------------------------
class GoFile:
    def __init__(self, path):
        self.src = open(path).read()
        self.toks = tokenize(self.src)
        self.vars = {}     # package-level name -> AST
        self.funcs = {}    # helper name -> (params, return AST)
        self.tests = {}    # TestName -> token index of body start
        self._scan()

    def _scan(self):
        t = self.toks
        i = 0
        depth = 0
        while t[i][0] != "eof":
            tok = t[i]
            if depth == 0 and tok == ("id", "func"):
                name = t[i + 1][1]
                if t[i + 1][1] == "(":  # method
                    i += 1
                    continue
                p = Parser(t, i + 2)
                params = self._params(p)
                while p.peek()[1] != "{":
                    p.next()
                body_start = p.i
                if name.startswith("Test") or re.match(r"test[A-Z]", name):
                    self.tests[name] = body_start
                else:
                    ret = self._single_return(body_start)
                    if ret is not None:
                        self.funcs[name] = (params, ret)
                p.skip_block()
                i = p.i
                continue
            if depth == 0 and tok == ("id", "var"):
                p = Parser(t, i + 1)
                if p.accept("("):
                    while not p.accept(")"):
                        if p.accept(";"):
                            continue
                        save = p.i
                        try:
                            self._var_spec(p)
                        except SyntaxError:
                            p.i = save
                            self._skip_stmt(p)
                else:
                    save = p.i
                    try:
                        self._var_spec(p)
                    except SyntaxError:
                        p.i = save
                        self._skip_stmt(p)
                i = p.i
                continue
            if tok[1] == "{":
                depth += 1
            elif tok[1] == "}":
                depth -= 1
            i += 1

    def _var_spec(self, p):
        names = [p.next()[1]]
        while p.accept(","):
            names.append(p.next()[1])
        if p.peek()[1] != "=":
            p.parse_type()
        if p.accept("="):
            vals = [p.parse_expr()]
            while p.accept(","):
                vals.append(p.parse_expr())
            for n, v in zip(names, vals):
                self.vars[n] = v
        p.accept(";")

    def _params(self, p):
        p.expect("(")
        names = []
        pending = []
        while not p.accept(")"):
            tok = p.next()
            if tok[1] == ",":
                continue
            if p.peek()[1] in (",", ")"):
                pending.append(tok[1])  # name in a grouped list (or a bare type)
                continue
            pending.append(tok[1])
            p.parse_type()
            names.extend(pending)
            pending = []
        return names

    def _single_return(self, body_start):
        p = Parser(self.toks, body_start)
        p.expect("{")
        if p.peek() == ("id", "return"):
            p.next()
            try:
                e = p.parse_expr()
            except SyntaxError:
                return None
            p.accept(";")
            if p.peek()[1] == "}":
                return e
        return None

    def test_locals_and_table(self, test, table="tests"):
        """Locals assigned (:=) in `test` before `<table> :=`, and the table's AST."""
        p = Parser(self.toks, self.tests[test])
        p.expect("{")
        local = {}
        while True:
            tok = p.peek()
            if tok[0] == "id" and p.peek(1)[1] in (":=", ","):
                save = p.i
                names = [p.next()[1]]
                while p.accept(","):
                    names.append(p.next()[1])
                if not p.accept(":="):
                    p.i = save
                    self._skip_stmt(p)
                    continue
                vals = [p.parse_expr()]
                while p.accept(","):
                    vals.append(p.parse_expr())
                if names == [table]:
                    return local, vals[0]
                for n, v in zip(names, vals):
                    local[n] = v
                p.accept(";")
            elif tok == ("id", "var"):
                p.next()
                names = [p.next()[1]]
                if p.peek()[1] != "=":
                    p.parse_type()
                if p.accept("="):
                    local[names[0]] = p.parse_expr()
                p.accept(";")
            elif tok[1] == ";":
                p.next()
            elif tok[1] == "}" or tok[0] == "eof":
                raise KeyError(f"{test}: no `{table} :=` table")
            else:
                self._skip_stmt(p)

    @staticmethod
    def _skip_stmt(p):
        """Skip to the end of the current statement (the next `;` at bracket depth 0)."""
        depth = 0
        while True:
            tok = p.next()
            if tok[0] == "eof":
                p.i -= 1
                return
            if tok[1] in ("{", "(", "["):
                depth += 1
            elif tok[1] in ("}", ")", "]"):
                depth -= 1
                if depth < 0:
                    p.i -= 1
                    return
            elif depth == 0 and tok[1] == ";":
                return


# --------------------------------------------------------------------------------------
# evaluation into v1 JSON
# --------------------------------------------------------------------------------------
CONSTS = {
    "v1.DoNotSchedule": "DoNotSchedule", "v1.ScheduleAnyway": "ScheduleAnyway",
    "v1.NodeInclusionPolicyHonor": "Honor", "v1.NodeInclusionPolicyIgnore": "Ignore",
    "metav1.LabelSelectorOpIn": "In", "metav1.LabelSelectorOpNotIn": "NotIn",
    "metav1.LabelSelectorOpExists": "Exists", "metav1.LabelSelectorOpDoesNotExist": "DoesNotExist",
    "v1.NodeSelectorOpIn": "In", "v1.NodeSelectorOpNotIn": "NotIn", "v1.NodeSelectorOpExists": "Exists",
    "v1.NodeSelectorOpDoesNotExist": "DoesNotExist", "v1.NodeSelectorOpGt": "Gt", "v1.NodeSelectorOpLt": "Lt",
    "v1.TaintEffectNoSchedule": "NoSchedule", "v1.TaintEffectPreferNoSchedule": "PreferNoSchedule",
    "v1.TaintEffectNoExecute": "NoExecute", "v1.TolerationOpExists": "Exists", "v1.TolerationOpEqual": "Equal",
    "v1.LabelHostname": "kubernetes.io/hostname", "v1.LabelTopologyZone": "topology.kubernetes.io/zone",
    "v1.LabelTopologyRegion": "topology.kubernetes.io/region",
    "v1.LabelZoneFailureDomainStable": "topology.kubernetes.io/zone",
    "v1.LabelZoneRegionStable": "topology.kubernetes.io/region",
    "v1.LabelZoneFailureDomain": "failure-domain.beta.kubernetes.io/zone",
    "v1.LabelZoneRegion": "failure-domain.beta.kubernetes.io/region",
    "v1.TaintNodeUnschedulable": "node.kubernetes.io/unschedulable",
    "v1.DefaultHardPodAffinitySymmetricWeight": 1,
    "v1.ResourceCPU": "cpu", "v1.ResourceMemory": "memory", "v1.ResourcePods": "pods",
    "v1.ResourceEphemeralStorage": "ephemeral-storage",
    "fwk.Success": 0, "fwk.Error": 1, "fwk.Unschedulable": 2, "fwk.UnschedulableAndUnresolvable": 3,
    "fwk.Wait": 4, "fwk.Skip": 5, "fwk.Pending": 6,
    "config.ListDefaulting": "List", "config.SystemDefaulting": "System",
    "fwk.MaxNodeScore": 100, "framework.MaxNodeScore": 100, "fwk.MinNodeScore": 0,
    "st.PodAffinityWithRequiredReq": "req", "st.PodAffinityWithPreferredReq": "pref",
    "st.PodAffinityWithRequiredPreferredReq": "reqpref", "st.PodAntiAffinityWithRequiredReq": "req",
    "st.PodAntiAffinityWithPreferredReq": "pref", "st.PodAntiAffinityWithRequiredPreferredReq": "reqpref",
    "st.NilPodAffinity": "nil", "st.NodeSelectorTypeMatchExpressions": "expr", "st.NodeSelectorTypeMatchFields": "fields",
    "v1.ResourceHugePagesPrefix": "hugepages-", "resource.DecimalSI": "DecimalSI", "resource.BinarySI": "BinarySI",
    "v1.ContainerRestartPolicyAlways": "Always",
    "config.LeastAllocated": "LeastAllocated", "config.MostAllocated": "MostAllocated",
    "config.RequestedToCapacityRatio": "RequestedToCapacityRatio",
    "true": True, "false": False, "nil": None,
}
PAUSE = "registry.k8s.io/pause:3.10.2"  # imageutils.GetPauseImageName (test/utils/image/manifest.go:233)


def go_sprintf(fmt, *args):
    out, i = [], 0
    k = 0
    while k < len(fmt):
        if fmt[k] == "%" and k + 1 < len(fmt):
            verb = fmt[k + 1]
            if verb == "%":
                out.append("%")
            else:
                out.append(str(args[i]))
                i += 1
            k += 2
        else:
            out.append(fmt[k])
            k += 1
    return "".join(out)


class Unknown(Exception):
    pass


_QSUFFIX = {"n": (10, -9), "u": (10, -6), "m": (10, -3), "": (10, 0), "k": (10, 3), "M": (10, 6), "G": (10, 9),
            "T": (10, 12), "P": (10, 15), "E": (10, 18), "Ki": (2, 10), "Mi": (2, 20), "Gi": (2, 30), "Ti": (2, 40),
            "Pi": (2, 50), "Ei": (2, 60)}


def quantity_value(q, milli=False):
    """resource.Quantity's Value() / MilliValue() of a canonical quantity string: the exact amount,
    rounded up (apimachinery/pkg/api/resource/quantity.go ScaledValue rounds toward +infinity)."""
    from fractions import Fraction
    m = re.fullmatch(r"([+-]?[0-9.]+)(?:[eE]([+-]?\d+)|(Ki|Mi|Gi|Ti|Pi|Ei|[numkMGTPE])?)", q.strip())
    if not m:
        raise Unknown(f"quantity {q!r}")
    v = Fraction(m.group(1))
    if m.group(2) is not None:
        v *= Fraction(10) ** int(m.group(2))
    else:
        base, exp = _QSUFFIX[m.group(3) or ""]
        v *= Fraction(base) ** exp
    if milli:
        v *= 1000
    return -((-v.numerator) // v.denominator)


def lower_camel(name):
    if name.isupper():
        return name.lower()
    m = re.match(r"^([A-Z]+)([A-Z][a-z].*)$", name)
    if m:  # HostIP -> hostIP ; URLPath -> urlPath
        return m.group(1).lower() + m.group(2)
    return name[:1].lower() + name[1:]


FIELD_MAP = {"ObjectMeta": "metadata", "TypeMeta": None}


class Status(dict):
    pass


MAP_TYPES = {"v1.ResourceList"}  # named map types: keys are expressions, not field names
# typed object literals (e.g. &appsv1.ReplicaSet{...} in a test's objs) -> (apiVersion, kind)
OBJECT_KINDS = {"v1.Service": ("v1", "Service"), "v1.ReplicationController": ("v1", "ReplicationController"),
                "appsv1.ReplicaSet": ("apps/v1", "ReplicaSet"), "appsv1.StatefulSet": ("apps/v1", "StatefulSet")}
GROUP_VERSIONS = {"appsv1.SchemeGroupVersion": "apps/v1", "v1.SchemeGroupVersion": "v1"}


class Evaluator:
    def __init__(self, gofile, extra_consts=None, helpers=None):
        self.f = gofile
        self.consts = dict(CONSTS)
        self.consts.update(extra_consts or {})
        self.helpers = dict(helpers or {})  # Python restatements of multi-statement test helpers

    def ev(self, e, env):
        k = e[0]
        if k == "lit":
            return e[1]
        if k == "id":
            name = e[1]
            if name in env:
                return self.ev(env[name], env) if isinstance(env[name], tuple) else env[name]
            if name in self.f.vars:
                return self.ev(self.f.vars[name], {})
            if name in self.consts:
                return self.consts[name]
            raise Unknown(name)
        if k == "sel":
            try:
                name = _dotted(e)
            except ValueError:
                name = None
            if name is not None and name in self.consts:
                return self.consts[name]
            base = self.ev(e[1], env)
            if isinstance(base, dict):
                return base.get(lower_camel(e[2]))
            raise Unknown(name or e[2])
        if k == "addr":
            return self.ev(e[1], env)
        if k == "deref":
            return self.ev(e[1], env)
        if k == "neg":
            return -self.ev(e[1], env)
        if k == "not":
            return not self.ev(e[1], env)
        if k == "bin":
            a, b = self.ev(e[2], env), self.ev(e[3], env)
            op = e[1]
            if op == "+":
                return a + b
            if op == "-":
                return a - b
            if op == "*":
                return a * b
            if op == "/":
                return a // b if isinstance(a, int) and isinstance(b, int) else a / b
            if op == "%":
                return a % b
            if op == "<<":
                return a << b
            raise Unknown(op)
        if k == "composite":
            return self.composite(e[1], e[2], env)
        if k == "elided":
            return self.composite(None, e[1], env)
        if k == "call":
            return self.call(e[1], [a for a in e[2]], env)
        if k == "index":
            base = self.ev(e[1], env)
            return base[self.ev(e[2], env)]
        raise Unknown(str(e[0]))

    def composite(self, typ, elems, env):
        kind = typ[0] if typ else None
        if kind == "slice" or kind == "array":
            inner = typ[-1]
            return [self.composite(inner, v[1], env) if v[0] == "elided" else self.ev(v, env) for _, v in elems]
        if kind == "map" or (kind == "named" and typ[1] in MAP_TYPES):
            if kind == "named":
                typ = ("map", None, ("named", "resource.Quantity"))
            out = {}
            for key, v in elems:
                kk = self.ev(key, env)
                out[kk] = self.composite(typ[2], v[1], env) if v[0] == "elided" else self.ev(v, env)
            return out
        if kind == "ptr":
            return self.composite(typ[1], elems, env)
        if kind == "named" and typ[1] in ("resource.Quantity",):
            raise Unknown("quantity literal")
        # struct-like: keys are field names
        out = {}
        for key, v in elems:
            if key is None:
                raise Unknown("positional struct literal")
            fname = key[1] if key[0] == "id" else _dotted(key)
            if typ is not None and kind == "map":
                pass
            jname = FIELD_MAP.get(fname, lower_camel(fname)) if fname in FIELD_MAP else lower_camel(fname)
            if jname is None:
                continue
            val = self.composite(None, v[1], env) if v[0] == "elided" else self.ev(v, env)
            out[jname] = val
        if kind == "named" and typ[1] in ("fwk.NodeScore", "framework.NodeScore"):
            return {"name": out.get("name"), "score": out.get("score", 0)}
        if kind == "named" and typ[1] in OBJECT_KINDS:  # runtime.Object literals keep their kind
            api, k = OBJECT_KINDS[typ[1]]
            out = dict(out, apiVersion=api, kind=k)
        return out

    def call(self, fn, args, env):
        if fn[0] == "index":  # explicit type arguments (ptr.To[int64](0), sets.New[string](...))
            return self.call(fn[1], args, env)
        # builder method call?
        if fn[0] == "sel":
            name = None
            try:
                name = _dotted(fn)
            except ValueError:
                pass
            if name in ("st.MakePod",):
                return PodB()
            if name in ("st.MakeNode",):
                return NodeB()
            if name in ("st.MakeLabelSelector",):
                return LSB()
            if name in ("ptr.To", "resource.MustParse", "int64", "int32", "int", "v1.ResourceName", "string"):
                return self.ev(args[0], env)
            if name is not None and name.endswith(".WithKind") and name[:-len(".WithKind")] in GROUP_VERSIONS:
                # schema.GroupVersion.WithKind -> GroupVersionKind
                return {"apiVersion": GROUP_VERSIONS[name[:-len(".WithKind")]], "kind": self.ev(args[0], env)}
            if name == "fmt.Sprintf":
                vals = [self.ev(a, env) for a in args]
                return go_sprintf(*vals)
            if name == "resource.NewMilliQuantity":
                return f"{self.ev(args[0], env)}m"
            if name == "resource.NewQuantity":
                return str(self.ev(args[0], env))
            if name in ("framework.NewNodeInfo",):
                return {"_nodeinfo_pods": [self.ev(a, env) for a in args]}
            if name in self.helpers:
                return self.helpers[name](*[self.ev(a, env) for a in args])
            if name in ("fwk.NewStatus", "framework.NewStatus"):
                vals = [self.ev(a, env) for a in args]
                return Status(code=vals[0], reasons=vals[1:])
            if name in ("fwk.AsStatus",):
                return Status(code=1, reasons=[])
            if fn[2] in ("MilliValue", "Value") and not args:  # resource.Quantity methods on a parsed quantity
                q = self.ev(fn[1], env)
                if isinstance(q, (str, int)):
                    return quantity_value(str(q), milli=fn[2] == "MilliValue")
            recv = self.ev(fn[1], env) if name is None or not name.split(".")[0] in ("st", "ptr", "fwk") else None
            if recv is None and name is not None and name.split(".")[0] in self.consts_pkgs():
                raise Unknown(name)
            if isinstance(recv, Builder):
                vals = [self.ev(a, env) for a in args]
                return recv.method(fn[2], vals)
            raise Unknown(name or fn[2])
        if fn[0] == "id":
            name = fn[1]
            if name in ("new",):
                return {}
            if name in ("int64", "int32", "int", "float64", "string"):
                return self.ev(args[0], env)
            if name in self.helpers:
                return self.helpers[name](*[self.ev(a, env) for a in args])
            if name in self.f.funcs:
                params, body = self.f.funcs[name]
                sub = dict(env)
                for pn, a in zip(params, args):
                    sub[pn] = self.ev(a, env)
                return self.ev(body, sub)
            if name == "append":
                base = list(self.ev(args[0], env) or [])
                for a in args[1:]:
                    v = self.ev(a, env)
                    base.extend(v if isinstance(v, list) else [v])
                return base
            raise Unknown(name)
        if fn[0] == "type":
            return self.ev(args[0], env)
        raise Unknown(str(fn))

    @staticmethod
    def consts_pkgs():
        return {"v1", "metav1", "fwk", "framework", "st", "ptr", "resource", "config", "schema"}


# --------------------------------------------------------------------------------------
# builders with the semantics of pkg/scheduler/testing/wrappers.go
# --------------------------------------------------------------------------------------
class Builder:
    def method(self, name, args):
        fn = getattr(self, "m_" + name, None)
        if fn is None:
            raise Unknown(f"{type(self).__name__}.{name}")
        return fn(*args)


class LSB(Builder):
    def __init__(self):
        self.o = {}

    def m_Label(self, k, v):
        self.o.setdefault("matchLabels", {})[k] = v
        return self

    def _expr(self, k, op, vals=None):
        e = {"key": k, "operator": op}
        if vals is not None:
            e["values"] = list(vals)
        self.o.setdefault("matchExpressions", []).append(e)
        return self

    def m_In(self, k, vals):
        return self._expr(k, "In", vals)

    def m_NotIn(self, k, vals):
        return self._expr(k, "NotIn", vals)

    def m_Exists(self, k):
        return self._expr(k, "Exists")

    def m_NotExist(self, k):
        return self._expr(k, "DoesNotExist")

    def m_Obj(self):
        return self.o


class NodeB(Builder):
    def __init__(self):  # MakeNode() = Capacity(nil): pods=32 allocatable
        self.o = {"apiVersion": "v1", "kind": "Node", "metadata": {}, "spec": {},
                  "status": {"capacity": {"pods": "32"}, "allocatable": {"pods": "32"}}}

    def m_Name(self, s):
        self.o["metadata"]["name"] = s
        return self

    def m_UID(self, s):
        self.o["metadata"]["uid"] = s
        return self

    def m_Label(self, k, v):
        self.o["metadata"].setdefault("labels", {})[k] = v
        return self

    def m_Capacity(self, res):
        r = {"pods": "32"}
        r.update({k: str(v) for k, v in (res or {}).items()})
        self.o["status"]["capacity"] = dict(r)
        self.o["status"]["allocatable"] = dict(r)
        return self

    def m_Taints(self, taints):
        self.o["spec"]["taints"] = taints
        return self

    def m_Unschedulable(self, v):
        self.o["spec"]["unschedulable"] = v
        return self

    def m_Images(self, images):
        self.o["status"]["images"] = [{"names": [n], "sizeBytes": s} for n, s in images.items()]
        return self

    def m_Obj(self):
        return self.o


class PodB(Builder):
    def __init__(self):
        self.o = {"apiVersion": "v1", "kind": "Pod", "metadata": {}, "spec": {"containers": []}}

    def m_Name(self, s):
        self.o["metadata"]["name"] = s
        return self

    def m_UID(self, s):
        self.o["metadata"]["uid"] = s
        return self

    def m_Namespace(self, s):
        self.o["metadata"]["namespace"] = s
        return self

    def m_Label(self, k, v):
        self.o["metadata"].setdefault("labels", {})[k] = v
        return self

    def m_Labels(self, d):
        for k, v in (d or {}).items():
            self.m_Label(k, v)
        return self

    def m_Node(self, s):
        self.o["spec"]["nodeName"] = s
        return self

    def m_Terminating(self):
        self.o["metadata"]["deletionTimestamp"] = "2024-01-01T00:00:00Z"
        return self

    def m_Priority(self, p):
        self.o["spec"]["priority"] = p
        return self

    def m_NominatedNodeName(self, n):  # wrappers.go: Status.NominatedNodeName
        self.o.setdefault("status", {})["nominatedNodeName"] = n
        return self

    def m_OwnerReference(self, name, gvk):  # wrappers.go:353-363: a controller reference
        self.o["metadata"]["ownerReferences"] = [{"apiVersion": gvk["apiVersion"], "kind": gvk["kind"],
                                                   "name": name, "controller": True}]
        return self

    def m_Toleration(self, key):
        self.o["spec"].setdefault("tolerations", []).append({"key": key, "operator": "Exists"})
        return self

    def m_Tolerations(self, ts):
        self.o["spec"]["tolerations"] = ts
        return self

    def m_NodeSelector(self, m):
        self.o["spec"]["nodeSelector"] = m
        return self

    def _na(self):
        return self.o["spec"].setdefault("affinity", {}).setdefault("nodeAffinity", {})

    def m_NodeAffinityIn(self, key, vals, t="expr"):
        term = ({"matchFields": [{"key": key, "operator": "In", "values": list(vals)}]} if t == "fields"
                else {"matchExpressions": [{"key": key, "operator": "In", "values": list(vals)}]})
        self._na()["requiredDuringSchedulingIgnoredDuringExecution"] = {"nodeSelectorTerms": [term]}
        return self

    def m_NodeAffinityNotIn(self, key, vals):
        term = {"matchExpressions": [{"key": key, "operator": "NotIn", "values": list(vals)}]}
        self._na()["requiredDuringSchedulingIgnoredDuringExecution"] = {"nodeSelectorTerms": [term]}
        return self

    def _pa(self, which, topo, sel, kind):
        if kind == "nil":
            return self
        pa = self.o["spec"].setdefault("affinity", {}).setdefault(which, {})
        term = {"labelSelector": sel, "topologyKey": topo}
        if kind in ("req", "reqpref"):
            pa.setdefault("requiredDuringSchedulingIgnoredDuringExecution", []).append(term)
        if kind in ("pref", "reqpref"):
            pa.setdefault("preferredDuringSchedulingIgnoredDuringExecution", []).append(
                {"weight": 1, "podAffinityTerm": term})
        return self

    def m_PodAffinity(self, topo, sel, kind):
        return self._pa("podAffinity", topo, sel, kind)

    def m_PodAntiAffinity(self, topo, sel, kind):
        return self._pa("podAntiAffinity", topo, sel, kind)

    def m_PodAffinityExists(self, k, topo, kind):
        return self._pa("podAffinity", topo, {"matchExpressions": [{"key": k, "operator": "Exists"}]}, kind)

    def m_PodAntiAffinityExists(self, k, topo, kind):
        return self._pa("podAntiAffinity", topo, {"matchExpressions": [{"key": k, "operator": "Exists"}]}, kind)

    def m_PodAffinityNotExists(self, k, topo, kind):
        return self._pa("podAffinity", topo, {"matchExpressions": [{"key": k, "operator": "DoesNotExist"}]}, kind)

    def m_PodAntiAffinityNotExists(self, k, topo, kind):
        return self._pa("podAntiAffinity", topo, {"matchExpressions": [{"key": k, "operator": "DoesNotExist"}]},
                        kind)

    def m_PodAffinityIn(self, k, topo, vals, kind):
        return self._pa("podAffinity", topo, {"matchExpressions": [{"key": k, "operator": "In", "values": list(vals)}]},
                        kind)

    def m_PodAntiAffinityIn(self, k, topo, vals, kind):
        return self._pa("podAntiAffinity", topo,
                        {"matchExpressions": [{"key": k, "operator": "In", "values": list(vals)}]}, kind)

    def m_PodAffinityNotIn(self, k, topo, vals, kind):
        return self._pa("podAffinity", topo,
                        {"matchExpressions": [{"key": k, "operator": "NotIn", "values": list(vals)}]}, kind)

    def m_PodAntiAffinityNotIn(self, k, topo, vals, kind):
        return self._pa("podAntiAffinity", topo,
                        {"matchExpressions": [{"key": k, "operator": "NotIn", "values": list(vals)}]}, kind)

    def m_SpreadConstraint(self, max_skew, key, when, sel, min_domains, aff_policy, taint_policy, mlk):
        c = {"maxSkew": max_skew, "topologyKey": key, "whenUnsatisfiable": when}
        if sel is not None:
            c["labelSelector"] = sel
        if min_domains is not None:
            c["minDomains"] = min_domains
        if aff_policy is not None:
            c["nodeAffinityPolicy"] = aff_policy
        if taint_policy is not None:
            c["nodeTaintsPolicy"] = taint_policy
        if mlk is not None:
            c["matchLabelKeys"] = list(mlk)
        self.o["spec"].setdefault("topologySpreadConstraints", []).append(c)
        return self

    def m_Req(self, req):  # wrappers.go:814-822
        if req:
            n = len(self.o["spec"]["containers"])
            self.o["spec"]["containers"].append({"name": f"con{n}", "image": PAUSE,
                                                 "resources": {"requests": {k: str(v) for k, v in req.items()}}})
        return self

    def m_InitReq(self, req):  # :836-844 (Resources: requests and limits)
        if req:
            ic = self.o["spec"].setdefault("initContainers", [])
            r = {k: str(v) for k, v in req.items()}
            ic.append({"name": f"init-con{len(ic)}", "image": PAUSE, "resources": {"requests": r, "limits": dict(r)}})
        return self

    def m_SidecarReq(self, req):  # :847-855
        if req:
            ic = self.o["spec"].setdefault("initContainers", [])
            r = {k: str(v) for k, v in req.items()}
            ic.append({"name": f"sidecar-con{len(ic)}", "image": PAUSE, "restartPolicy": "Always",
                       "resources": {"requests": r, "limits": dict(r)}})
        return self

    def m_Container(self, image):  # :366-370
        n = len(self.o["spec"]["containers"])
        self.o["spec"]["containers"].append({"name": f"con{n}", "image": image})
        return self

    def m_Containers(self, cs):
        self.o["spec"]["containers"] = list(cs)
        return self

    def m_Overhead(self, rl):
        self.o["spec"]["overhead"] = {k: str(v) for k, v in rl.items()}
        return self

    def m_Resources(self, rr):  # pod-level resources (:339-342)
        self.o["spec"]["resources"] = rr
        return self

    def m_Obj(self):
        return self.o


def load_table(path, test, table="tests", extra_consts=None, helpers=None):
    """-> list of dicts (field name -> evaluated value or Unknown marker)."""
    import glob
    import os
    gf = GoFile(path)
    for sib in sorted(glob.glob(os.path.join(os.path.dirname(path), "*_test.go"))):  # same package
        if sib != path:
            o = GoFile(sib)
            for k, v in o.vars.items():
                gf.vars.setdefault(k, v)
            for k, v in o.funcs.items():
                gf.funcs.setdefault(k, v)
    local, tab = gf.test_locals_and_table(test, table)
    ev = Evaluator(gf, extra_consts, helpers)
    env = dict(local)
    assert tab[0] == "composite", tab[0]
    out = []
    for _, elem in tab[2]:
        assert elem[0] == "elided"
        case = {}
        bad = None
        for key, v in elem[1]:
            fname = key[1]
            try:
                case[fname] = ev.composite(None, v[1], env) if v[0] == "elided" else ev.ev(v, env)
            except (Unknown, KeyError, TypeError) as ex:
                bad = f"{fname}: {ex}"
        case["_unsupported"] = bad
        out.append(case)
    return out, gf
