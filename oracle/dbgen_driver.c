/*
 * Driver over the reference's vendored TPC-H dbgen (third_party/tpch-dbgen, compiled where it lies by
 * oracle/Makefile `ref`; never copied). Generates CUSTOMER, then ORDERS and LINEITEM exactly as the reference's
 * TpchDbGenerator::generate does (src/benchmarklib/tpch/tpch_db_generator.cpp:203-236: dbgen_reset_seeds, then per
 * row row_start / mk_cust or mk_order / row_stop, money through convert_money) and prints the columns the hot-path
 * fixtures use as tab-separated text:
 *   C <c_custkey> <c_mktsegment>
 *   O <o_orderkey> <o_custkey> <o_orderdate> <o_shippriority>
 *   L <l_orderkey> <l_quantity> <l_extendedprice> <l_discount> <l_tax> <l_returnflag> <l_linestatus> <l_shipdate>
 * Floats are printed with %.9g (round-trips float32).
 * usage: dbgen_driver <scale factor>
 */
#include <stdio.h>
#include <stdlib.h>

#include "dss.h"
#include "dsstypes.h"
#include "tpch_dbgen.h"

/* tpch_db_generator.cpp:148-152 */
static float convert_money(DSS_HUGE cents) {
  const DSS_HUGE dollars = cents / 100;
  cents %= 100;
  return dollars + ((float)cents) / 100.0f;
}

int main(int argc, char** argv) {
  const float sf = argc > 1 ? (float)atof(argv[1]) : 0.01f;
  static order_t order;
  static customer_t cust;
  dbgen_reset_seeds();
  /* tpch_db_generator.cpp:206-214 */
  const size_t customer_count = (size_t)(tdefs[CUST].base * sf);
  for (size_t i = 0; i < customer_count; ++i) {
    row_start(CUST);
    mk_cust((DSS_HUGE)(i + 1), &cust);
    row_stop(CUST);
    printf("C\t%lld\t%s\n", (long long)cust.custkey, cust.mktsegment);
  }
  const size_t order_count = (size_t)(tdefs[ORDER].base * sf);
  for (size_t i = 0; i < order_count; ++i) {
    row_start(ORDER);
    mk_order((DSS_HUGE)(i + 1), &order, 0l, sf);
    row_stop(ORDER);
    printf("O\t%lld\t%lld\t%s\t%lld\n", (long long)order.okey, (long long)order.custkey, order.odate,
           (long long)order.spriority);
    for (int l = 0; l < (int)order.lines; ++l) {
      const line_t* li = &order.l[l];
      printf("L\t%lld\t%.9g\t%.9g\t%.9g\t%.9g\t%c\t%c\t%s\n", (long long)li->okey, (double)(float)li->quantity,
             (double)convert_money(li->eprice), (double)convert_money(li->discount), (double)convert_money(li->tax),
             li->rflag[0], li->lstatus[0], li->sdate);
    }
  }
  return 0;
}
