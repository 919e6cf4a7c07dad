// A small DOM for running the website's ES modules under node in tests: elements with attributes, classes, styles,
// children, events, value/checked, textContent, and querySelector(All) for '#id', '.cls', 'tag', '[attr=v]'
// compounds and descendant chains. Plus fetch over node's http module, history/location, localStorage and
// timers — enough for the packages' components to render and talk to a live control plane.
import http from 'http';

class Node_ {
    constructor() {
        this.parentNode = null;
        this.childNodes = [];
    }
    get firstChild() {
        return this.childNodes[0] || null;
    }
    appendChild(c) {
        if (c.parentNode) c.parentNode.removeChild(c);
        c.parentNode = this;
        this.childNodes.push(c);
        return c;
    }
    removeChild(c) {
        const i = this.childNodes.indexOf(c);
        if (i >= 0) this.childNodes.splice(i, 1);
        c.parentNode = null;
        return c;
    }
    remove() {
        if (this.parentNode) this.parentNode.removeChild(this);
    }
    get textContent() {
        return this.childNodes.map(c => c.textContent).join('');
    }
    set textContent(v) {
        this.childNodes = [];
        if (v !== '' && v !== null && v !== undefined) this.appendChild(new Text_(String(v)));
    }
}

class Text_ extends Node_ {
    constructor(t) {
        super();
        this.data = t;
        this.nodeType = 3;
    }
    get textContent() {
        return this.data;
    }
    set textContent(v) {
        this.data = String(v);
    }
}

class ClassList {
    constructor(el) {
        this.el = el;
    }
    _get() {
        return (this.el.getAttribute('class') || '').split(/\s+/).filter(Boolean);
    }
    contains(c) {
        return this._get().includes(c);
    }
    add(c) {
        const s = this._get();
        if (!s.includes(c)) s.push(c);
        this.el.setAttribute('class', s.join(' '));
    }
    remove(c) {
        this.el.setAttribute('class', this._get().filter(x => x !== c).join(' '));
    }
    toggle(c, on) {
        const want = on === undefined ? !this.contains(c) : !!on;
        if (want) this.add(c);
        else this.remove(c);
        return want;
    }
}

function parseSimple(sel) {
    // tag#id.cls[attr=value] — one compound selector
    const out = { tag: null, id: null, classes: [], attrs: [] };
    const re = /([a-zA-Z0-9_-]+)|#([a-zA-Z0-9_-]+)|\.([a-zA-Z0-9_-]+)|\[([a-zA-Z0-9_-]+)(?:=["']?([^\]"']*)["']?)?\]/g;
    let m;
    while ((m = re.exec(sel))) {
        if (m[1]) out.tag = m[1].toLowerCase();
        else if (m[2]) out.id = m[2];
        else if (m[3]) out.classes.push(m[3]);
        else out.attrs.push([m[4], m[5]]);
    }
    return out;
}

function matchesSimple(el, s) {
    if (!(el instanceof Element_)) return false;
    if (s.tag && el.tagName.toLowerCase() !== s.tag) return false;
    if (s.id && el.getAttribute('id') !== s.id) return false;
    for (const c of s.classes) if (!el.classList.contains(c)) return false;
    for (const [a, v] of s.attrs) {
        if (!el.hasAttribute(a)) return false;
        if (v !== undefined && el.getAttribute(a) !== v) return false;
    }
    return true;
}

function matches(el, selector) {
    const parts = selector.trim().split(/\s+/).map(parseSimple);
    if (!matchesSimple(el, parts[parts.length - 1])) return false;
    let k = parts.length - 2;
    let p = el.parentNode;
    while (k >= 0 && p) {
        if (matchesSimple(p, parts[k])) k--;
        p = p.parentNode;
    }
    return k < 0;
}

class Element_ extends Node_ {
    constructor(tag, ns) {
        super();
        this.tagName = tag.toUpperCase();
        this.namespaceURI = ns || null;
        this.attributes = {};
        this.listeners = {};
        this.style = {};
        this.classList = new ClassList(this);
        this._value = '';
        this.checked = false;
        this.disabled = false;
        this.hidden = false;
        this.nodeType = 1;
        this.selectionStart = 0;
        this.selectionEnd = 0;
    }
    get className() {
        return this.getAttribute('class') || '';
    }
    set className(v) {
        this.setAttribute('class', v);
    }
    get id() {
        return this.getAttribute('id') || '';
    }
    get value() {
        if (this.tagName === 'SELECT' && this._value === '') {
            const opts = this.querySelectorAll('option');
            const sel = opts.find(o => o.hasAttribute('selected')) || opts[0];
            return sel ? sel.value : '';
        }
        if (this.tagName === 'OPTION' && this._value === '') return this.getAttribute('value') || this.textContent;
        return this._value;
    }
    set value(v) {
        this._value = String(v);
    }
    setAttribute(k, v) {
        this.attributes[k] = String(v);
    }
    getAttribute(k) {
        return Object.prototype.hasOwnProperty.call(this.attributes, k) ? this.attributes[k] : null;
    }
    hasAttribute(k) {
        return Object.prototype.hasOwnProperty.call(this.attributes, k);
    }
    removeAttribute(k) {
        delete this.attributes[k];
    }
    addEventListener(type, fn) {
        (this.listeners[type] = this.listeners[type] || []).push(fn);
    }
    dispatch(type, extra) {
        const ev = Object.assign({ type, target: this, preventDefault() {}, stopPropagation() {} }, extra || {});
        let n = this;
        while (n) {
            for (const fn of (n.listeners && n.listeners[type]) || []) fn(ev);
            n = n.parentNode;
        }
        return ev;
    }
    click() {
        return this.dispatch('click');
    }
    // set a form control's value and fire the event the components listen to
    input(v) {
        if (this.getAttribute('type') === 'checkbox') {
            this.checked = !!v;
            return this.dispatch('change');
        }
        this.value = v;
        return this.dispatch(this.tagName === 'SELECT' ? 'change' : 'input');
    }
    closest(sel) {
        let n = this;
        while (n && n instanceof Element_) {
            if (matches(n, sel)) return n;
            n = n.parentNode;
        }
        return null;
    }
    querySelectorAll(sel) {
        const out = [];
        const alts = sel.split(',');
        const walk = n => {
            for (const c of n.childNodes) {
                if (c instanceof Element_) {
                    if (alts.some(a => matches(c, a))) out.push(c);
                    walk(c);
                }
            }
        };
        walk(this);
        return out;
    }
    querySelector(sel) {
        return this.querySelectorAll(sel)[0] || null;
    }
    get innerText() {
        return this.textContent;
    }
}

export function installDom(baseUrl) {
    const body = new Element_('body');
    const document = {
        body,
        createElement: t => new Element_(t),
        createElementNS: (ns, t) => new Element_(t, ns),
        createTextNode: t => new Text_(t),
        getElementById: id => body.querySelector('#' + id),
        addEventListener() {},
        querySelector: s => body.querySelector(s),
        querySelectorAll: s => body.querySelectorAll(s)
    };
    const store = {};
    const location = { pathname: '/', href: baseUrl + '/' };
    global.document = document;
    global.location = location;
    global.history = {
        pushState: (a, b, p) => (location.pathname = p),
        replaceState: (a, b, p) => (location.pathname = p)
    };
    global.window = {
        localStorage: {
            getItem: k => (k in store ? store[k] : null),
            setItem: (k, v) => (store[k] = String(v)),
            removeItem: k => delete store[k]
        },
        addEventListener() {}
    };
    global.performance = global.performance || { now: () => Date.now() };
    global.URLSearchParams = URLSearchParams;
    global.fetch = (url, opts) =>
        new Promise((resolve, reject) => {
            opts = opts || {};
            const u = new URL(url, baseUrl);
            const req = http.request(u, { method: opts.method || 'GET', headers: opts.headers || {} }, res => {
                let data = '';
                res.setEncoding('utf8');
                res.on('data', d => (data += d));
                res.on('end', () =>
                    resolve({ ok: res.statusCode < 400, status: res.statusCode, text: async () => data, json: async () => JSON.parse(data) })
                );
            });
            req.on('error', reject);
            if (opts.body) req.write(opts.body);
            req.end();
        });
    return document;
}

export const sleep = ms => new Promise(r => setTimeout(r, ms));

export async function waitFor(fn, ms) {
    const end = Date.now() + (ms || 5000);
    for (;;) {
        const v = fn();
        if (v) return v;
        if (Date.now() > end) throw new Error('timed out waiting: ' + fn.toString());
        await sleep(20);
    }
}

export function buttonByText(root, text) {
    return root.querySelectorAll('button').find(b => b.textContent.trim() === text) || null;
}
