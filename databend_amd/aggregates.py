"""Aggregate-function descriptors: the host mirror of `AggregateFunctionFactory` / `AggregateFunction`.

The reference resolves `factory.get(name, params, arguments)` into an `AggregateFunctionRef`
(FUN/aggregate_function_factory.rs:157-220): the named function, wrapped by
`AggregateFunctionCombinatorNull` when an argument is nullable and by
`AggregateFunctionOrNullAdaptor` unless the function returns a default for empty input (count).
The GPU path identifies each function by exactly that triple: its kind,
its argument DataType and the or_null wrapping.  `return_type()` is answered by the C ABI
(`dbg_agg_result_type`) so the host mirror and the kernels cannot disagree.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Sequence

from . import abi
from .column import DataType

# "sql_avg": SQL's avg(x), which the planner rewrites to sum(x) / if(count(x) = 0, 1, count(x))
# (SQL/planner/semantic/aggregate_rewriter.rs:145-208), fused into one aggregate whose finalize
# does the division (DBG_AGG_AVG_SQL); "avg" is AggregateAvgFunction itself (FUN/aggregate_avg.rs).
_KINDS = {"count": abi.AGG_COUNT, "sum": abi.AGG_SUM, "min": abi.AGG_MIN, "max": abi.AGG_MAX,
          "avg": abi.AGG_AVG, "sql_avg": abi.AGG_AVG_SQL}


@dataclass(frozen=True)
class AggregateFunction:
    """An `AggregateFunctionRef` as the GPU path sees it."""
    display_name: str
    kind: int
    arg: Optional[DataType]  # None => count(*)
    or_null: bool = True
    # AggregateDistinctCombinator over the nested kind (suffix "_distinct",
    # FUN/aggregate_combinator_distinct.rs): run by databend_amd.distinct.DistinctAggregator
    distinct: bool = False

    def name(self) -> str:
        # AggregateCountFunction reports its struct name (FUN/aggregate_count.rs:69-71)
        return "AggregateCountFunction" if self.kind == abi.AGG_COUNT else self.display_name

    def to_abi(self) -> abi.dbg_agg_spec:
        if self.distinct:
            from .ffi import Unsupported
            raise Unsupported(abi.DBG_ERR_UNSUPPORTED, f"{self.display_name}: a DISTINCT aggregate is not one table "
                              "state; run it with databend_amd.distinct.DistinctAggregator")
        s = abi.dbg_agg_spec()
        s.kind = self.kind
        if self.arg is None:
            s.arg = abi.dbg_datatype(-1, 0, 0, 0, 0)
        else:
            s.arg = self.arg.to_abi()
        s.or_null = 1 if (self.or_null and self.kind != abi.AGG_COUNT) else 0
        return s

    def return_type(self) -> DataType:
        from .ffi import lib, check
        if self.distinct:  # the combinator returns the nested function's type (:60-62)
            from dataclasses import replace
            return replace(self, distinct=False, arg=self.arg.wrap_nullable() if self.arg else None).return_type()
        out = abi.dbg_datatype()
        spec = self.to_abi()
        check(lib().dbg_agg_result_type(abi.C.byref(spec), abi.C.byref(out)))
        return DataType.from_abi(out)


class AggregateFunctionFactory:
    """`AggregateFunctionFactory::instance().get(name, params, arguments)` for the GPU path's set."""

    _inst = None

    @classmethod
    def instance(cls) -> "AggregateFunctionFactory":
        if cls._inst is None:
            cls._inst = cls()
        return cls._inst

    def get(self, name: str, params: Sequence = (), arguments: Sequence[DataType] = ()) -> AggregateFunction:
        return self.get_or_null(name, params, arguments, True)

    def get_or_null(self, name: str, params: Sequence, arguments: Sequence[DataType], or_null: bool) -> AggregateFunction:
        lname = name.lower()
        distinct = lname.endswith("_distinct") and lname != "sql_avg_distinct"
        if distinct:  # the combinator suffix (FUN/aggregate_function_factory.rs: combinator_desc)
            lname = lname[: -len("_distinct")]
            if not arguments:
                raise ValueError(f"{name} requires an argument")
        if lname not in _KINDS:
            raise NotImplementedError(f"Unsupported AggregateFunction on the GPU path: {name}")
        if len(arguments) > 1:
            raise NotImplementedError(f"{name}: only unary aggregates are on the GPU path")
        arg = arguments[0] if arguments else None
        if lname != "count" and arg is None:
            raise ValueError(f"{name} requires one argument")
        return AggregateFunction(name, _KINDS[lname], arg, or_null, distinct)
