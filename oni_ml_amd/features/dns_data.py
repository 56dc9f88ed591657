"""Reference data for the DNS featurizer.

COUNTRY_CODES: the ccTLD set the domain parser tests the last label against
(dns_pre_lda.scala:180, dns_post_lda.scala:148).  The reference's set also
contains the empty string, which can never match a last label once Java's
split has dropped trailing empty labels; it is kept for fidelity.
SPECIAL_DOMAIN: the domain flagged top_domain = 2 (dns_pre_lda.scala:315).
"""

COUNTRY_CODES = tuple((
    "ac ad ae af ag ai al am an ao aq ar as at au aw ax az ba bb bd be bf bg bh bi bj bm bn bo bq br "
    "bs bt bv bw by bz ca cc cd cf cg ch ci ck cl cm cn co cr cu cv cw cx cy cz de dj dk dm do dz ec "
    "ee eg eh er es et eu fi fj fk fm fo fr ga gb gd ge gf gg gh gi gl gm gn gp gq gr gs gt gu gw gy "
    "hk hm hn hr ht hu id ie il im in io iq ir is it je jm jo jp ke kg kh ki km kn kp kr krd kw ky kz "
    "la lb lc li lk lr ls lt lu lv ly ma mc md me mg mh mk ml mm mn mo mp mq mr ms mt mu mv mw mx my "
    "mz na nc ne nf ng ni nl no np nr nu nz om pa pe pf pg ph pk pl pm pn pr ps pt pw py qa re ro rs "
    "ru rw sa sb sc sd se sg sh si sj sk sl sm sn so sr ss st su sv sx sy sz tc td tf tg th tj tk tl "
    "tm tn to tp tr tt tv tw tz ua ug uk us uy uz va vc ve vg vi vn vu wf ws ye yt za zm zw "
).split()) + ("",)

SPECIAL_DOMAIN = "intel"
